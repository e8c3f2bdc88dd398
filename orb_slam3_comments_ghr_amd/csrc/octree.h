// octree.h — ORBextractor::DistributeOctTree (ref:src/ORBextractor.cc:716-1050) on the host, for
// osg_orb_detect (fast.hip).  Host-only C++ (no HIP types), so it also builds in a plain g++ harness.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

namespace osg_oct {

// ---- DistributeOctTree (ref:src/ORBextractor.cc:716-1050) on the host ------------------------------
// Nodes live in a pool and form a doubly linked list in the reference's list order; a node's
// keypoints are a range of an index pool (DivideNode copies them to its children in order).
struct Key4 {  // a keypoint as the kernels write it: (x, y, response, unused); plain host struct
    float x, y, z, w;
};

struct OctNode {
    int ulx, uly, urx, ury, blx, bly, brx, bry;
    int kbeg, kcnt;
    bool no_more;
    int prev, next;
};

struct OctTree {
    const Key4 *keys;
    std::vector<OctNode> nodes;
    std::vector<int> kidx;
    std::vector<uint8_t> qbuf;  // DivideNode's quadrant per keypoint (scratch)
    int head = -1, size = 0;

    int new_node()
    {
        nodes.push_back(OctNode{});
        OctNode &n = nodes.back();
        n.prev = n.next = -1;
        n.no_more = false;
        return (int)nodes.size() - 1;
    }
    void push_front(int id)
    {
        nodes[id].prev = -1;
        nodes[id].next = head;
        if (head >= 0) nodes[head].prev = id;
        head = id;
        size++;
    }
    void push_back_after(int tail, int id)
    {
        nodes[id].prev = tail;
        nodes[id].next = -1;
        if (tail >= 0) nodes[tail].next = id;
        else head = id;
        size++;
    }
    int erase(int id)  // returns the next node
    {
        const int p = nodes[id].prev, n = nodes[id].next;
        if (p >= 0) nodes[p].next = n;
        else head = n;
        if (n >= 0) nodes[n].prev = p;
        size--;
        return n;
    }
    // ExtractorNode::DivideNode (:607-654): the four children's geometry and keypoints (in the
    // parent's order), pushed to the list front as the caller does (n1, n2, n3, n4, non-empty
    // only); children with > 1 keypoint are appended to `expand`
    void divide(int id, std::vector<std::pair<int, int>> &expand, int *n_expand)
    {
        const OctNode P = nodes[id];
        const int halfX = (int)std::ceil(static_cast<float>(P.urx - P.ulx) / 2);
        const int halfY = (int)std::ceil(static_cast<float>(P.bry - P.uly) / 2);
        int ch[4];
        for (int q = 0; q < 4; q++) ch[q] = new_node();
        OctNode *c = &nodes[0];
        OctNode &n1 = c[ch[0]], &n2 = c[ch[1]], &n3 = c[ch[2]], &n4 = c[ch[3]];
        n1.ulx = P.ulx, n1.uly = P.uly, n1.urx = P.ulx + halfX, n1.ury = P.uly;
        n1.blx = P.ulx, n1.bly = P.uly + halfY, n1.brx = P.ulx + halfX, n1.bry = P.uly + halfY;
        n2.ulx = n1.urx, n2.uly = n1.ury, n2.urx = P.urx, n2.ury = P.ury;
        n2.blx = n1.brx, n2.bly = n1.bry, n2.brx = P.urx, n2.bry = P.uly + halfY;
        n3.ulx = n1.blx, n3.uly = n1.bly, n3.urx = n1.brx, n3.ury = n1.bry;
        n3.blx = P.blx, n3.bly = P.bly, n3.brx = n1.brx, n3.bry = P.bly;
        n4.ulx = n3.urx, n4.uly = n3.ury, n4.urx = n2.brx, n4.ury = n2.bry;
        n4.blx = n3.brx, n4.bly = n3.bry, n4.brx = P.brx, n4.bry = P.bry;
        // classify into four runs of the index pool, each in the parent's order
        int cnt[4] = {0, 0, 0, 0};
        std::vector<uint8_t> &q = qbuf;
        q.resize(P.kcnt);
        for (int k = 0; k < P.kcnt; k++) {
            const Key4 kp = keys[kidx[P.kbeg + k]];
            const int qq = (kp.x < n1.urx) ? ((kp.y < n1.bry) ? 0 : 2) : ((kp.y < n1.bry) ? 1 : 3);
            q[k] = (uint8_t)qq;
            cnt[qq]++;
        }
        int beg[4];
        beg[0] = (int)kidx.size();
        for (int t = 1; t < 4; t++) beg[t] = beg[t - 1] + cnt[t - 1];
        kidx.resize(kidx.size() + P.kcnt);
        int fill[4] = {beg[0], beg[1], beg[2], beg[3]};
        for (int k = 0; k < P.kcnt; k++) kidx[fill[q[k]]++] = kidx[P.kbeg + k];
        for (int t = 0; t < 4; t++) {
            OctNode &n = nodes[ch[t]];
            n.kbeg = beg[t];
            n.kcnt = cnt[t];
            n.no_more = cnt[t] == 1;
            if (cnt[t] > 0) {
                push_front(ch[t]);
                if (cnt[t] > 1) {
                    if (n_expand) (*n_expand)++;
                    expand.push_back(std::make_pair(cnt[t], ch[t]));
                }
            }
        }
    }
};

// keys[0 .. nk) in vToDistributeKeys order (relative to (minX, minY)); out: the kept keypoints
void distribute_oct_tree(const Key4 *keys, int nk, int minX, int maxX, int minY, int maxY, int N,
                         std::vector<Key4> &out)
{
    out.clear();
    // per host thread, kept across calls: fresh multi-MB vectors per call cost more in page faults
    // than the whole tree walk
    thread_local OctTree T;
    T.keys = keys;
    T.nodes.clear();
    T.kidx.clear();
    T.head = -1;
    T.size = 0;
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
    const float hX = static_cast<float>(maxX - minX) / nIni;
    std::vector<int> ini(nIni);
    int tail = -1;
    for (int i = 0; i < nIni; i++) {
        const int id = T.new_node();
        OctNode &n = T.nodes[id];
        n.ulx = (int)(hX * static_cast<float>(i));
        n.uly = 0;
        n.urx = (int)(hX * static_cast<float>(i + 1));
        n.ury = 0;
        n.blx = n.ulx;
        n.bly = maxY - minY;
        n.brx = n.urx;
        n.bry = maxY - minY;
        T.push_back_after(tail, id);
        tail = id;
        ini[i] = id;
    }
    // keypoints to the initial nodes (:739-745), in order
    std::vector<int> cnt(nIni, 0), which(nk);
    for (int k = 0; k < nk; k++) {
        which[k] = (int)(keys[k].x / hX);
        cnt[which[k]]++;
    }
    int off = 0;
    for (int i = 0; i < nIni; i++) {
        T.nodes[ini[i]].kbeg = off;
        T.nodes[ini[i]].kcnt = 0;
        off += cnt[i];
    }
    T.kidx.resize(nk);
    for (int k = 0; k < nk; k++) {
        OctNode &n = T.nodes[ini[which[k]]];
        T.kidx[n.kbeg + n.kcnt++] = k;
    }
    for (int id = T.head; id >= 0;) {
        OctNode &n = T.nodes[id];
        if (n.kcnt == 1) {
            n.no_more = true;
            id = n.next;
        } else if (n.kcnt == 0)
            id = T.erase(id);
        else
            id = n.next;
    }
    bool finish = false;
    std::vector<std::pair<int, int>> expand, prev;
    auto cmp = [&](const std::pair<int, int> &a, const std::pair<int, int> &b) {  // compareNodes (:656-676)
        if (a.first < b.first) return true;
        if (a.first > b.first) return false;
        return T.nodes[a.second].ulx < T.nodes[b.second].ulx;
    };
    while (!finish) {
        const int prevSize = T.size;
        int nToExpand = 0;
        expand.clear();
        for (int id = T.head; id >= 0;) {
            if (T.nodes[id].no_more) {
                id = T.nodes[id].next;
                continue;
            }
            T.divide(id, expand, &nToExpand);
            id = T.erase(id);
        }
        if (T.size >= N || T.size == prevSize) {
            finish = true;
        } else if (T.size + nToExpand * 3 > N) {
            while (!finish) {
                const int prevSize2 = T.size;
                prev = expand;
                expand.clear();
                std::sort(prev.begin(), prev.end(), cmp);
                for (int j = (int)prev.size() - 1; j >= 0; j--) {
                    T.divide(prev[j].second, expand, nullptr);
                    T.erase(prev[j].second);
                    if (T.size >= N) break;
                }
                if (T.size >= N || T.size == prevSize2) finish = true;
            }
        }
    }
    // the strongest keypoint of every node, first maximum, in list order (:1033-1048)
    for (int id = T.head; id >= 0; id = T.nodes[id].next) {
        const OctNode &n = T.nodes[id];
        int best = T.kidx[n.kbeg];
        float r = keys[best].z;
        for (int k = 1; k < n.kcnt; k++) {
            const int kk = T.kidx[n.kbeg + k];
            if (keys[kk].z > r) {
                best = kk;
                r = keys[kk].z;
            }
        }
        out.push_back(keys[best]);
    }
}


}  // namespace osg_oct
