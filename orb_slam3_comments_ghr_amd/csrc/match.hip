// match.hip — placeholder (filled in next)
#include "osg_internal.h"
#include "match_common.h"
extern "C" {
int osg_search_by_projection_mps(osg_ctx *ctx, const osg_frame *, const osg_mp_queries *, float, float, int, float, int32_t *, const uint8_t *) { return osg_set_error(ctx, OSG_E_UNSUPPORTED, "not built"); }
int osg_search_by_projection_last(osg_ctx *ctx, const osg_frame *, const osg_last_queries *, float, int, int, int32_t *, const uint8_t *) { return osg_set_error(ctx, OSG_E_UNSUPPORTED, "not built"); }
int osg_search_by_projection_kf(osg_ctx *ctx, const osg_frame *, const osg_kf_queries *, float, int, int, int32_t *) { return osg_set_error(ctx, OSG_E_UNSUPPORTED, "not built"); }
int osg_search_by_bow_kf_f(osg_ctx *ctx, const osg_bow_side *, const osg_bow_side *, float, int, int32_t *) { return osg_set_error(ctx, OSG_E_UNSUPPORTED, "not built"); }
int osg_search_by_bow_kf_kf(osg_ctx *ctx, const osg_bow_side *, const osg_bow_side *, float, int, int32_t *) { return osg_set_error(ctx, OSG_E_UNSUPPORTED, "not built"); }
}
