/* oracle_desc.c — CPU restatement of MapPoint::ComputeDistinctiveDescriptors (ref:src/MapPoint.cc:444-535).
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
 * Per MapPoint: the float Distances[N][N] matrix of DescriptorDistance, each row copied to a
 * vector<int>, std::sort, element [0.5 * (N - 1)], and the first row with the smallest such
 * median.  best_idx = -1 when the point has no descriptor (the reference returns early). */
#include <stdlib.h>

#include "oracle.h"

static int cmp_int(const void *a, const void *b)
{
    const int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

void oracle_compute_distinctive_descriptors(const uint8_t *desc, const int32_t *start, int n_points, int32_t *best_idx)
{
    for (int p = 0; p < n_points; p++) {
        const size_t N = (size_t)(start[p + 1] - start[p]);
        const uint8_t *D = desc + 32 * (size_t)start[p];
        best_idx[p] = -1;
        if (N == 0) continue;                                  /* :479-480 */
        float *Distances = (float *)malloc(sizeof(float) * N * N);
        int *vDists = (int *)malloc(sizeof(int) * N);
        for (size_t i = 0; i < N; i++) {                       /* :487-498 */
            Distances[i * N + i] = 0;
            for (size_t j = i + 1; j < N; j++) {
                const int distij = oracle_descriptor_distance(D + 32 * i, D + 32 * j);
                Distances[i * N + j] = (float)distij;
                Distances[j * N + i] = (float)distij;
            }
        }
        int BestMedian = 0x7FFFFFFF, BestIdx = 0;               /* :502-520 */
        for (size_t i = 0; i < N; i++) {
            for (size_t j = 0; j < N; j++) vDists[j] = (int)Distances[i * N + j];
            qsort(vDists, N, sizeof(int), cmp_int);
            const int median = vDists[(size_t)(0.5 * (double)(N - 1))];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = (int)i;
            }
        }
        best_idx[p] = BestIdx;
        free(Distances);
        free(vDists);
    }
}
