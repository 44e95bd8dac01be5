// Test scaffold: stands where the reference's src/defs.h sits in its tree.  The reference's
// defs.h pulls in Eigen and OpenCV (absent from this image); this one provides the pr:: types of
// the facade's POD branch, so the mock tree below compiles the way the reference's does.
#pragma once
#include "pr/defs.h"
