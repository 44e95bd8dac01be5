// Replaces the reference's src/camera.h (llepa/02-VisualOdometry) in its source tree: pr::Camera
// becomes the facade's value type (same constructor, projectPoint/projectPoints and pose
// accessors), which the device solver marshals.  Included by name from src/picp_solver.h and
// src/cam.h:7.  Build recipe: INTEGRATION.md §2.
#pragma once
#include "defs.h"
#include "pr/camera.h"
