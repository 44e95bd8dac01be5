// Replaces the reference's src/picp_solver.h (llepa/02-VisualOdometry) in its source tree:
// pr::PICPSolver becomes the MI355X facade over libpicp_amd.so.  The reference's own
// src/cam.h:6, src/my_utilities.h:23 and src/cam.cpp:4 include this file by that name, so the
// swap needs no edit to any caller.  Build recipe: INTEGRATION.md §2.
#pragma once
#include "defs.h"          // the reference's src/defs.h (Eigen + OpenCV typedefs), as before
#include "pr/picp_solver.h"
