// launchers for APAD = 8 (see mgn_launch.h)
#include "mgn_launch_impl.h"
MGN_DEFINE_APAD(8)
