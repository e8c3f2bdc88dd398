/* osg_dbow.h — DBoW2 vocabulary transform on gfx950.
 *
 * Replaces TemplatedVocabulary<FORB::TDescriptor, FORB>::transform(features, BowVector&,
 * FeatureVector&, levelsup) (ref:Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1192, descent
 * :1214-1256) as called by Frame::ComputeBoW (ref:src/Frame.cc:995-1010, levelsup = 4) and
 * KeyFrame::ComputeBoW.  The FeatureVector comes out as the CSR osg_featvec that
 * osg_search_by_bow_* consume.  No CPU fallback. */
#ifndef OSG_DBOW_H
#define OSG_DBOW_H
#include <stdint.h>

#include "osg.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { OSG_W_TF_IDF = 0, OSG_W_TF = 1, OSG_W_IDF = 2, OSG_W_BINARY = 3 };          /* DBoW2 WeightingType */
enum { OSG_S_L1 = 0, OSG_S_L2 = 1, OSG_S_CHI2 = 2, OSG_S_KL = 3, OSG_S_BHATT = 4, OSG_S_DOT = 5 }; /* ScoringType */

/* A vocabulary as TemplatedVocabulary::loadFromTextFile leaves it in memory
 * (ref:Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1334-1415): node 0 is the root; nodes 1..n-1
 * in file order, each with its parent, leaf flag, 32-byte descriptor and weight.  A node's children
 * are the nodes naming it as parent, in id order; leaves get word ids 0, 1, ... in id order. */
typedef struct osg_vocabulary_desc {
    int32_t k, L;                 /* branching factor, depth levels */
    int32_t scoring, weighting;   /* OSG_S_*, OSG_W_* */
    int32_t n_nodes;              /* including the root */
    const int32_t *parent;        /* n_nodes (parent[0] unused) */
    const uint8_t *is_leaf;       /* n_nodes */
    const uint8_t *desc;          /* n_nodes x 32 (the root's unused) */
    const double *weight;         /* n_nodes */
} osg_vocabulary_desc;

/* BowVector (std::map<WordId, WordValue>) as ascending arrays, and FeatureVector
 * (std::map<NodeId, vector<unsigned>>) as CSR.  Capacities: n_features entries each, node_start
 * n_features + 1. */
typedef struct osg_bow_out {
    int32_t n_words;              /* out */
    int32_t *word;
    double *value;
    int32_t n_nodes;              /* out */
    uint32_t *node_id;
    int32_t *node_start;
    int32_t *feat;
} osg_bow_out;

typedef struct osg_vocabulary osg_vocabulary;

/* Upload a vocabulary to the context's device (breadth-first renumbered so that a node's children
 * are consecutive).  k <= 32. */
int osg_vocabulary_create(osg_ctx *ctx, const osg_vocabulary_desc *v, osg_vocabulary **out);
/* Parse a DBoW2 text vocabulary (ORBvoc.txt format) and upload it. */
int osg_vocabulary_load_text(osg_ctx *ctx, const char *path, osg_vocabulary **out);
int osg_vocabulary_destroy(osg_vocabulary *voc);
/* Sizes of a loaded vocabulary: out4 = {k, L, n_nodes, n_words}. */
int osg_vocabulary_info(const osg_vocabulary *voc, int32_t *out4);

/* transform(features, BowVector, FeatureVector, levelsup) of one descriptor set (n x 32 bytes, the
 * rows of Frame::mDescriptors in order). */
int osg_vocabulary_transform(osg_ctx *ctx, const osg_vocabulary *voc, const uint8_t *desc, int32_t n,
                             int32_t levelsup, osg_bow_out *out);
/* B descriptor sets in one launch: set b has n[b] rows starting at row sum(n[0..b)) of desc;
 * out[b] as above. */
int osg_vocabulary_transform_batch(osg_ctx *ctx, const osg_vocabulary *voc, const uint8_t *desc,
                                   const int32_t *n, int32_t B, int32_t levelsup, osg_bow_out *out);

#ifdef __cplusplus
}
#endif
#endif /* OSG_DBOW_H */
