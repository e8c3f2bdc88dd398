/* oracle_dbow.c — CPU restatement of DBoW2's TemplatedVocabulary::transform(features, BowVector,
 * FeatureVector, levelsup) for ORB descriptors (FORB).  TEST INFRASTRUCTURE ONLY: the checker for
 * tests/, never linked into the product.
 *
 *   descent        ref:Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1214-1256 (strict '<': the
 *                  first child in children order wins ties; nid = node at level L - levelsup)
 *   distance       ref:Thirdparty/DBoW2/DBoW2/FORB.cpp:92-111 (8 x int32 SWAR popcount)
 *   BowVector      addWeight (TF, TF_IDF) / addIfNotExist (IDF, BINARY) in feature order,
 *                  ref:Thirdparty/DBoW2/DBoW2/BowVector.cpp:35-59; stopped words (weight <= 0)
 *                  are skipped (:1158, :1183)
 *   normalisation  ref:TemplatedVocabulary.h:1163-1191 and BowVector.cpp:63-85; mustNormalize per
 *                  scoring type, ref:Thirdparty/DBoW2/DBoW2/ScoringObject.h:80-95
 *   FeatureVector  addFeature (push_back in feature order), ref:FeatureVector.cpp:32-46
 *   children order TemplatedVocabulary::loadFromTextFile, ref:TemplatedVocabulary.h:1334-1415
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int forb_distance(const uint8_t *a, const uint8_t *b)
{
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        int32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        unsigned int v = (unsigned int)(x ^ y);
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24);
    }
    return dist;
}

typedef struct {
    int n;
    int *child_start, *child; /* CSR, children in id order */
    int *word_of;             /* word id per node, -1 for internal nodes */
} voc_index;

static void voc_build(const osg_vocabulary_desc *V, voc_index *X)
{
    const int n = V->n_nodes;
    X->n = n;
    X->child_start = (int *)calloc((size_t)n + 1, sizeof(int));
    X->child = (int *)malloc(sizeof(int) * (size_t)(n > 1 ? n : 1));
    X->word_of = (int *)malloc(sizeof(int) * (size_t)n);
    for (int i = 1; i < n; i++) X->child_start[V->parent[i] + 1]++;
    for (int i = 0; i < n; i++) X->child_start[i + 1] += X->child_start[i];
    int *fill = (int *)malloc(sizeof(int) * (size_t)n);
    memcpy(fill, X->child_start, sizeof(int) * (size_t)n);
    for (int i = 1; i < n; i++) X->child[fill[V->parent[i]]++] = i;
    free(fill);
    int w = 0;
    X->word_of[0] = -1;
    for (int i = 1; i < n; i++) X->word_of[i] = V->is_leaf[i] ? w++ : -1;
}

static void voc_free(voc_index *X)
{
    free(X->child_start);
    free(X->child);
    free(X->word_of);
}

/* transform(feature, word_id, weight, &nid, levelsup), ref:TemplatedVocabulary.h:1214-1256 */
static void descend(const osg_vocabulary_desc *V, const voc_index *X, const uint8_t *f, int levelsup,
                    int *word, double *weight, int *nid)
{
    const int nid_level = V->L - levelsup;
    if (nid_level <= 0) *nid = 0;
    int final_id = 0, level = 0;
    do {
        ++level;
        const int s = X->child_start[final_id], e = X->child_start[final_id + 1];
        int best = X->child[s];
        double best_d = (double)forb_distance(f, V->desc + 32 * (size_t)best);
        for (int c = s + 1; c < e; c++) {
            const int id = X->child[c];
            const double d = (double)forb_distance(f, V->desc + 32 * (size_t)id);
            if (d < best_d) {
                best_d = d;
                best = id;
            }
        }
        final_id = best;
        if (level == nid_level) *nid = final_id;
    } while (!V->is_leaf[final_id]);
    *word = X->word_of[final_id];
    *weight = V->weight[final_id];
}

typedef struct {
    int key, idx;
    double w;
} kv;

static int kv_cmp(const void *a, const void *b)
{
    const kv *x = (const kv *)a, *y = (const kv *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

static void transform_one(const osg_vocabulary_desc *V, const voc_index *Xp, const uint8_t *desc, int n,
                          int levelsup, osg_bow_out *out)
{
    out->n_words = 0;
    out->n_nodes = 0;
    out->node_start[0] = 0;
    if (V->n_nodes <= 1 || n <= 0) return; /* empty(): ref:TemplatedVocabulary.h:1133-1136 */
    const voc_index X = *Xp;
    kv *bw = (kv *)malloc(sizeof(kv) * (size_t)n), *fv = (kv *)malloc(sizeof(kv) * (size_t)n);
    int m = 0;
    for (int i = 0; i < n; i++) {
        int word, nid = 0;
        double w;
        descend(V, &X, desc + 32 * (size_t)i, levelsup, &word, &w, &nid);
        if (w > 0) { /* not stopped */
            bw[m].key = word;
            bw[m].idx = i;
            bw[m].w = w;
            fv[m].key = nid;
            fv[m].idx = i;
            fv[m].w = 0;
            m++;
        }
    }
    qsort(bw, (size_t)m, sizeof(kv), kv_cmp);
    qsort(fv, (size_t)m, sizeof(kv), kv_cmp);
    /* BowVector: addWeight sums in feature order (TF, TF_IDF); addIfNotExist keeps the first */
    const int add = (V->weighting == OSG_W_TF || V->weighting == OSG_W_TF_IDF);
    int nw = 0;
    for (int j = 0; j < m; j++) {
        if (nw > 0 && out->word[nw - 1] == bw[j].key) {
            if (add) out->value[nw - 1] += bw[j].w;
        } else {
            out->word[nw] = bw[j].key;
            out->value[nw] = bw[j].w;
            nw++;
        }
    }
    out->n_words = nw;
    const int must = V->scoring != OSG_S_DOT;
    const int l2 = V->scoring == OSG_S_L2;
    if (add && nw > 0 && !must) {
        const double nd = (double)nw;
        for (int j = 0; j < nw; j++) out->value[j] /= nd;
    }
    if (must) {
        double norm = 0.0;
        if (!l2)
            for (int j = 0; j < nw; j++) norm += fabs(out->value[j]);
        else {
            for (int j = 0; j < nw; j++) norm += out->value[j] * out->value[j];
            norm = sqrt(norm);
        }
        if (norm > 0.0)
            for (int j = 0; j < nw; j++) out->value[j] /= norm;
    }
    /* FeatureVector */
    int nn = 0;
    for (int j = 0; j < m; j++) {
        if (!(nn > 0 && (int)out->node_id[nn - 1] == fv[j].key)) {
            out->node_id[nn] = (uint32_t)fv[j].key;
            out->node_start[nn] = j;
            nn++;
        }
        out->feat[j] = fv[j].idx;
    }
    out->node_start[nn] = m;
    out->n_nodes = nn;
    free(bw);
    free(fv);
}

void oracle_dbow_transform(const osg_vocabulary_desc *V, const uint8_t *desc, int n, int levelsup, osg_bow_out *out)
{
    voc_index X;
    voc_build(V, &X);
    transform_one(V, &X, desc, n, levelsup, out);
    voc_free(&X);
}

/* B sets with the children index built once, as the reference builds its tree once at load
 * (the CPU baseline's per-frame work) */
void oracle_dbow_transform_batch(const osg_vocabulary_desc *V, const uint8_t *desc, const int32_t *n, int B,
                                 int levelsup, osg_bow_out *out)
{
    voc_index X;
    voc_build(V, &X);
    size_t first = 0;
    for (int b = 0; b < B; b++) {
        transform_one(V, &X, desc + 32 * first, n[b], levelsup, &out[b]);
        first += (size_t)n[b];
    }
    voc_free(&X);
}
