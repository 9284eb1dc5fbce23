// launchers for APAD = 16 (see mgn_launch.h)
#include "mgn_launch_impl.h"
MGN_DEFINE_APAD(16)
