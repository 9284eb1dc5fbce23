// launchers for APAD = 1 (see mgn_launch.h)
#include "mgn_launch_impl.h"
MGN_DEFINE_APAD(1)
