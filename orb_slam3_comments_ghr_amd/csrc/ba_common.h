// ba_common.h — device helpers shared by the BA kernels.
#pragma once
