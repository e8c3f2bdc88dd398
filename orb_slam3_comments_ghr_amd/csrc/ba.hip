// ba.hip — placeholder (filled in next)
#include "osg_internal.h"
#include "ba_common.h"
extern "C" {
int osg_local_bundle_adjustment(osg_ctx *ctx, const osg_ba_graph *, osg_ba_result *, const volatile int *) { return osg_set_error(ctx, OSG_E_UNSUPPORTED, "not built"); }
}
