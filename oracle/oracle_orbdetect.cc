// oracle_orbdetect.cc — CPU restatement of ORBextractor::ComputeKeyPointsOctTree.
// TEST INFRASTRUCTURE ONLY: the checker for tests/, never linked into the product.
//  * The cell loop (ref:src/ORBextractor.cc:1065-1198): W = 35 cells over [minBorder, maxBorder)
//    (EDGE_THRESHOLD - 3 .. size - EDGE_THRESHOLD + 3), each cell FAST'd with iniThFAST and, when
//    that finds nothing, with minThFAST; cell keypoints shifted by (j wCell, i hCell).
//  * DistributeOctTree (ref:src/ORBextractor.cc:716-1050) with ExtractorNode::DivideNode (:607-654)
//    and compareNodes (:656-676), written with std::list / std::vector / std::sort exactly as the
//    reference holds them (push_front order, erase through the stored iterator, std::sort's order
//    for nodes of equal size and UL.x), so the output order is the reference's.
//  * Then pt += (minBorderX, minBorderY), octave = level, size = (int)(PATCH_SIZE * scale) (:1186-1196).
// cv::FAST is OpenCV's (not in the reference tree): its published algorithm (modules/features2d
// fast.cpp, FAST_t<16> with the 9-of-16 test, cornerScore<16> and the 3x3 strict-max non-maximum
// suppression, keypoints emitted row by row, response = score) is restated in fast_cell() below;
// parity with OpenCV itself is unpinned.  fast_cell() reads the cell as its own image, as the
// reference's rowRange / colRange ROI does: rows / cols 3 .. size - 4 are tested, neighbours outside
// the tested range have score 0 in the suppression.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <list>
#include <vector>

#include "oracle.h"

namespace {

struct Key {
    float x, y, response;
};

const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                            {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// cornerScore<16>: the largest threshold at which the pixel is still a 9-of-16 corner
int corner_score(const uint8_t *p, const int *pixel, int threshold)
{
    const int N = 25;
    int d[N];
    const int v = p[0];
    for (int k = 0; k < N; k++) d[k] = v - p[pixel[k]];
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], d[k + 2]);
        a = std::min(a, d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, d[k + 4]);
        a = std::min(a, d[k + 5]);
        a = std::min(a, d[k + 6]);
        a = std::min(a, d[k + 7]);
        a = std::min(a, d[k + 8]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(d[k + 1], d[k + 2]);
        b = std::max(b, d[k + 3]);
        b = std::max(b, d[k + 4]);
        b = std::max(b, d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, d[k + 6]);
        b = std::max(b, d[k + 7]);
        b = std::max(b, d[k + 8]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    return -b0 - 1;
}

// FAST_t<16>(img, keypoints, threshold, nonmax_suppression = true) on a rows x cols image with
// `step` bytes per row
void fast_cell(const uint8_t *img, int rows, int cols, int step, int threshold, std::vector<Key> &out)
{
    out.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    const int K = 8, N = 25;
    int pixel[N];
    for (int k = 0; k < 16; k++) pixel[k] = kCircle[k][0] + kCircle[k][1] * step;
    for (int k = 16; k < N; k++) pixel[k] = pixel[k - 16];
    uint8_t tab[512];
    for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (rows < 7 || cols < 7) return;
    std::vector<uint8_t> score((size_t)rows * cols, 0);
    for (int i = 3; i < rows - 3; i++) {
        const uint8_t *row = img + (size_t)i * step;
        for (int j = 3; j < cols - 3; j++) {
            const uint8_t *ptr = row + j;
            const int v = ptr[0];
            const uint8_t *t = tab - v + 255;
            int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
            if (d == 0) continue;
            d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
            d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
            d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
            if (d == 0) continue;
            d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
            d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
            d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
            d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
            bool corner = false;
            if (d & 1) {
                const int vt = v - threshold;
                int count = 0;
                for (int k = 0; k < N; k++) {
                    if (ptr[pixel[k]] < vt) {
                        if (++count > K) {
                            corner = true;
                            break;
                        }
                    } else
                        count = 0;
                }
            }
            if (!corner && (d & 2)) {
                const int vt = v + threshold;
                int count = 0;
                for (int k = 0; k < N; k++) {
                    if (ptr[pixel[k]] > vt) {
                        if (++count > K) {
                            corner = true;
                            break;
                        }
                    } else
                        count = 0;
                }
            }
            if (corner) score[(size_t)i * cols + j] = (uint8_t)corner_score(ptr, pixel, threshold);
        }
    }
    // strict 3 x 3 maximum, in row-major order
    for (int i = 3; i < rows - 3; i++)
        for (int j = 3; j < cols - 3; j++) {
            const int s = score[(size_t)i * cols + j];
            if (!s) continue;
            bool keep = true;
            for (int di = -1; di <= 1 && keep; di++)
                for (int dj = -1; dj <= 1; dj++) {
                    if (!di && !dj) continue;
                    if (!(s > score[(size_t)(i + di) * cols + j + dj])) {
                        keep = false;
                        break;
                    }
                }
            if (keep) out.push_back(Key{(float)j, (float)i, (float)s});
        }
}

struct Point2i {
    int x, y;
};

struct ExtractorNode {
    std::vector<Key> vKeys;
    Point2i UL, UR, BL, BR;
    std::list<ExtractorNode>::iterator lit;
    bool bNoMore = false;

    void DivideNode(ExtractorNode &n1, ExtractorNode &n2, ExtractorNode &n3, ExtractorNode &n4)
    {
        const int halfX = (int)std::ceil(static_cast<float>(UR.x - UL.x) / 2);
        const int halfY = (int)std::ceil(static_cast<float>(BR.y - UL.y) / 2);
        n1.UL = UL;
        n1.UR = Point2i{UL.x + halfX, UL.y};
        n1.BL = Point2i{UL.x, UL.y + halfY};
        n1.BR = Point2i{UL.x + halfX, UL.y + halfY};
        n2.UL = n1.UR;
        n2.UR = UR;
        n2.BL = n1.BR;
        n2.BR = Point2i{UR.x, UL.y + halfY};
        n3.UL = n1.BL;
        n3.UR = n1.BR;
        n3.BL = BL;
        n3.BR = Point2i{n1.BR.x, BL.y};
        n4.UL = n3.UR;
        n4.UR = n2.BR;
        n4.BL = n3.BR;
        n4.BR = BR;
        for (const Key &kp : vKeys) {
            if (kp.x < n1.UR.x) {
                if (kp.y < n1.BR.y) n1.vKeys.push_back(kp);
                else n3.vKeys.push_back(kp);
            } else if (kp.y < n1.BR.y)
                n2.vKeys.push_back(kp);
            else
                n4.vKeys.push_back(kp);
        }
        if (n1.vKeys.size() == 1) n1.bNoMore = true;
        if (n2.vKeys.size() == 1) n2.bNoMore = true;
        if (n3.vKeys.size() == 1) n3.bNoMore = true;
        if (n4.vKeys.size() == 1) n4.bNoMore = true;
    }
};

bool compareNodes(const std::pair<int, ExtractorNode *> &e1, const std::pair<int, ExtractorNode *> &e2)
{
    if (e1.first < e2.first) return true;
    if (e1.first > e2.first) return false;
    return e1.second->UL.x < e2.second->UL.x;
}

std::vector<Key> DistributeOctTree(const std::vector<Key> &vToDistributeKeys, int minX, int maxX, int minY, int maxY,
                                   int N)
{
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
    const float hX = static_cast<float>(maxX - minX) / nIni;
    std::list<ExtractorNode> lNodes;
    std::vector<ExtractorNode *> vpIniNodes(nIni);
    for (int i = 0; i < nIni; i++) {
        ExtractorNode ni;
        ni.UL = Point2i{(int)(hX * static_cast<float>(i)), 0};
        ni.UR = Point2i{(int)(hX * static_cast<float>(i + 1)), 0};
        ni.BL = Point2i{ni.UL.x, maxY - minY};
        ni.BR = Point2i{ni.UR.x, maxY - minY};
        lNodes.push_back(ni);
        vpIniNodes[i] = &lNodes.back();
    }
    for (const Key &kp : vToDistributeKeys) vpIniNodes[(int)(kp.x / hX)]->vKeys.push_back(kp);
    auto lit = lNodes.begin();
    while (lit != lNodes.end()) {
        if (lit->vKeys.size() == 1) {
            lit->bNoMore = true;
            lit++;
        } else if (lit->vKeys.empty())
            lit = lNodes.erase(lit);
        else
            lit++;
    }
    bool bFinish = false;
    std::vector<std::pair<int, ExtractorNode *>> vSizeAndPointerToNode;
    vSizeAndPointerToNode.reserve(lNodes.size() * 4);
    auto push_child = [&](ExtractorNode &c, int *nToExpand) {
        if (c.vKeys.size() > 0) {
            lNodes.push_front(c);
            if (c.vKeys.size() > 1) {
                if (nToExpand) (*nToExpand)++;
                vSizeAndPointerToNode.push_back(std::make_pair((int)c.vKeys.size(), &lNodes.front()));
                lNodes.front().lit = lNodes.begin();
            }
        }
    };
    while (!bFinish) {
        const int prevSize = (int)lNodes.size();
        lit = lNodes.begin();
        int nToExpand = 0;
        vSizeAndPointerToNode.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) {
                lit++;
                continue;
            }
            ExtractorNode n1, n2, n3, n4;
            lit->DivideNode(n1, n2, n3, n4);
            push_child(n1, &nToExpand);
            push_child(n2, &nToExpand);
            push_child(n3, &nToExpand);
            push_child(n4, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {
                const int prevSize2 = (int)lNodes.size();
                std::vector<std::pair<int, ExtractorNode *>> vPrevSizeAndPointerToNode = vSizeAndPointerToNode;
                vSizeAndPointerToNode.clear();
                std::sort(vPrevSizeAndPointerToNode.begin(), vPrevSizeAndPointerToNode.end(), compareNodes);
                for (int j = (int)vPrevSizeAndPointerToNode.size() - 1; j >= 0; j--) {
                    ExtractorNode n1, n2, n3, n4;
                    vPrevSizeAndPointerToNode[j].second->DivideNode(n1, n2, n3, n4);
                    push_child(n1, nullptr);
                    push_child(n2, nullptr);
                    push_child(n3, nullptr);
                    push_child(n4, nullptr);
                    lNodes.erase(vPrevSizeAndPointerToNode[j].second->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize2) bFinish = true;
            }
        }
    }
    std::vector<Key> vResultKeys;
    for (auto &node : lNodes) {
        const Key *pKP = &node.vKeys[0];
        float maxResponse = pKP->response;
        for (size_t k = 1; k < node.vKeys.size(); k++)
            if (node.vKeys[k].response > maxResponse) {
                pKP = &node.vKeys[k];
                maxResponse = node.vKeys[k].response;
            }
        vResultKeys.push_back(*pKP);
    }
    return vResultKeys;
}

}  // namespace

extern "C" int oracle_fast(const uint8_t *img, int rows, int cols, int step, int threshold, int cap, float *x, float *y,
                           float *response)
{
    std::vector<Key> k;
    fast_cell(img, rows, cols, step, threshold, k);
    if ((int)k.size() > cap) return -1;
    for (size_t i = 0; i < k.size(); i++) {
        x[i] = k[i].x;
        y[i] = k[i].y;
        response[i] = k[i].response;
    }
    return (int)k.size();
}

extern "C" int oracle_orb_detect(const osg_image_pyramid *P, int ini_th, int min_th, const int32_t *n_features,
                                 const float *scale_factors, int cap, float *x, float *y, float *response, float *size,
                                 int32_t *level_start)
{
    const int EDGE_THRESHOLD = 19, PATCH_SIZE = 31;
    const float W = 35;
    int total = 0;
    level_start[0] = 0;
    std::vector<Key> vKeysCell;
    for (int level = 0; level < P->n_levels; ++level) {
        const uint8_t *im = P->data[level];
        const int rows = P->rows[level], cols = P->cols[level], step = P->step[level];
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = cols - EDGE_THRESHOLD + 3, maxBorderY = rows - EDGE_THRESHOLD + 3;
        std::vector<Key> vToDistributeKeys;
        const float width = (maxBorderX - minBorderX), height = (maxBorderY - minBorderY);
        const int nCols = (int)(width / W), nRows = (int)(height / W);
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        for (int i = 0; i < nRows; i++) {
            const float iniY = minBorderY + i * hCell;
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = minBorderX + j * wCell;
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = maxBorderX;
                const int r0 = (int)iniY, r1 = (int)maxY, c0 = (int)iniX, c1 = (int)maxX;  // cv::Range(int, int)
                const uint8_t *sub = im + (size_t)r0 * step + c0;
                fast_cell(sub, r1 - r0, c1 - c0, step, ini_th, vKeysCell);
                if (vKeysCell.empty()) fast_cell(sub, r1 - r0, c1 - c0, step, min_th, vKeysCell);
                for (Key k : vKeysCell) {
                    k.x += j * wCell;
                    k.y += i * hCell;
                    vToDistributeKeys.push_back(k);
                }
            }
        }
        std::vector<Key> keys =
            DistributeOctTree(vToDistributeKeys, minBorderX, maxBorderX, minBorderY, maxBorderY, n_features[level]);
        const int scaledPatchSize = (int)(PATCH_SIZE * scale_factors[level]);
        if (total + (int)keys.size() > cap) return -1;
        for (const Key &k : keys) {
            x[total] = k.x + minBorderX;
            y[total] = k.y + minBorderY;
            response[total] = k.response;
            size[total] = (float)scaledPatchSize;
            total++;
        }
        level_start[level + 1] = total;
    }
    return total;
}
