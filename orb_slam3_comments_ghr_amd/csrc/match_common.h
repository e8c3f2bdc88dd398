// match_common.h — device helpers shared by the matcher kernels.
#pragma once
