// host_san.hip — the host runtime of liborbslam3_amd under AddressSanitizer / ThreadSanitizer, on the CPU
// (audit the launch path's host code for r04's SIGSEGV).  No GPU call is made: the
// driver exercises what the LBA / BA host path does between launches and what several host threads
// share —
//   * build_structure (ba.hip) on 8 threads at once, window path and map path (the worker pool's
//     thread_local scratch vectors), every graph's hash equal to its single-threaded build;
//   * osg_parallel_for (runtime.hip's process-wide worker pool) under 8..24 concurrent callers;
//   * osg_packer::fill_parallel (match_common.h: the pinned-block packer the LBA upload uses).
// Built by tools/sanitize/run.sh with runtime.hip compiled into the same executable (sanitized too);
// graphs come as arrays files written by tools/sanitize/run.py.
#include "../micro/lba_host_time.hip"
#include "../micro/packer_check.hip"

#include <cstdio>
#include <fstream>
#include <iterator>
#include <unordered_map>

namespace {
struct GraphBuf {
    std::vector<double> pose, point, obs;
    std::vector<uint8_t> fixed;
    std::vector<int32_t> e_point, e_pose, e_cam;
    std::vector<int8_t> e_kind;
    std::vector<float> isig;
    std::vector<osg_camera> cams;
    osg_ba_graph g{};
};
// tools/adapter_arrays.py's file format: {u32 name_len, name, u8 dtype, u64 count, data} repeated
using Arrays = std::unordered_map<std::string, std::vector<unsigned char>>;
Arrays read_arrays(const char *path)
{
    std::ifstream f(path, std::ios::binary);
    const std::vector<unsigned char> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    Arrays m;
    size_t o = 0;
    while (o + 4 <= d.size()) {
        uint32_t n;
        std::memcpy(&n, &d[o], 4);
        o += 4;
        const std::string name((const char *)&d[o], n);
        o += n;
        const char t = (char)d[o++];
        uint64_t cnt;
        std::memcpy(&cnt, &d[o], 8);
        o += 8;
        const size_t sz = cnt * (t == 'b' ? 1 : t == 'd' ? 8 : 4);
        m[name].assign(d.begin() + o, d.begin() + o + sz);
        o += sz;
    }
    return m;
}
template <class T>
std::vector<T> vec(const Arrays &m, const std::string &k)
{
    const std::vector<unsigned char> &a = m.at(k);
    std::vector<T> v(a.size() / sizeof(T));
    std::memcpy(v.data(), a.data(), a.size());
    return v;
}
GraphBuf load_graph(const char *path)
{
    const Arrays m = read_arrays(path);
    GraphBuf b;
    b.pose = vec<double>(m, "pose");
    b.point = vec<double>(m, "point");
    b.obs = vec<double>(m, "e_obs");
    b.fixed = vec<uint8_t>(m, "pose_fixed");
    b.e_point = vec<int32_t>(m, "e_point");
    b.e_pose = vec<int32_t>(m, "e_pose");
    b.e_cam = vec<int32_t>(m, "e_cam");
    b.e_kind = vec<int8_t>(m, "e_kind");
    b.isig = vec<float>(m, "e_inv_sigma2");
    const std::vector<uint8_t> cb = vec<uint8_t>(m, "cams");
    b.cams.resize(cb.size() / sizeof(osg_camera));
    std::memcpy(b.cams.data(), cb.data(), cb.size());
    osg_ba_graph &g = b.g;
    g.n_poses = (int)b.fixed.size();
    g.pose = b.pose.data();
    g.pose_fixed = b.fixed.data();
    g.n_points = (int)(b.point.size() / 3);
    g.point = b.point.data();
    g.n_edges = (int)b.e_point.size();
    g.e_point = b.e_point.data();
    g.e_pose = b.e_pose.data();
    g.e_kind = b.e_kind.data();
    g.e_cam = b.e_cam.data();
    g.e_obs = b.obs.data();
    g.e_inv_sigma2 = b.isig.data();
    g.n_cams = (int)b.cams.size();
    g.cams = b.cams.data();
    g.iterations = 10;
    return b;
}
}  // namespace

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: host_san graph.arrays...\n");
        return 2;
    }
    std::vector<GraphBuf> G;
    for (int i = 1; i < argc; i++) G.push_back(load_graph(argv[i]));
    for (auto &b : G) {  // the vectors moved: re-point the graph structs
        osg_ba_graph &g = b.g;
        g.pose = b.pose.data(); g.pose_fixed = b.fixed.data(); g.point = b.point.data();
        g.e_point = b.e_point.data(); g.e_pose = b.e_pose.data(); g.e_kind = b.e_kind.data();
        g.e_cam = b.e_cam.data(); g.e_obs = b.obs.data(); g.e_inv_sigma2 = b.isig.data(); g.cams = b.cams.data();
    }
    int fails = 0;
    for (int mode = 0; mode < 2; mode++) {
        if (mode) setenv("OSG_LBA_MAP_MODE", "1", 1);
        std::vector<unsigned long long> want(G.size());
        for (size_t i = 0; i < G.size(); i++) want[i] = lba_host_struct_hash(&G[i].g);
        std::vector<std::thread> th;
        std::atomic<int> bad{0};
        for (size_t i = 0; i < 8; i++)
            th.emplace_back([&, i] {
                for (int r = 0; r < 3; r++)
                    if (lba_host_struct_hash(&G[(i + r) % G.size()].g) != want[(i + r) % G.size()]) bad++;
            });
        for (auto &t : th) t.join();
        printf("structure build, %s path, 8 threads x 3: %d mismatches\n", mode ? "map" : "window", bad.load());
        fails += bad.load();
    }
    for (int T : {8, 24}) {
        const int b = pool_stress(T, 60, 333);
        printf("worker pool, %d concurrent callers: %d wrong sums\n", T, b);
        fails += b;
    }
    {
        std::vector<std::thread> th;
        std::atomic<int> bad{0};
        for (int t = 0; t < 4; t++)
            th.emplace_back([&, t] { bad += packer_check(100 + t, 12, 8) != 0; });
        for (auto &t : th) t.join();
        printf("packer fill_parallel, 4 concurrent packers: %d failures\n", bad.load());
        fails += bad.load();
    }
    printf("%s\n", fails ? "FAIL" : "OK");
    return fails ? 1 : 0;
}
