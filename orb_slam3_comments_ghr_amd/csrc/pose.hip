// pose.hip — placeholder (filled in next)
#include "osg_internal.h"
#include "ba_common.h"
extern "C" {
int osg_pose_optimization(osg_ctx *ctx, const osg_pose_problem *, osg_pose_result *) { return osg_set_error(ctx, OSG_E_UNSUPPORTED, "not built"); }
int osg_pose_optimization_batch(osg_ctx *ctx, const osg_pose_problem *, int32_t, osg_pose_result *) { return osg_set_error(ctx, OSG_E_UNSUPPORTED, "not built"); }
}
