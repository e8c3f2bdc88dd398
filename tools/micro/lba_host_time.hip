// Host-only timing of the LBA structure build (ba.hip's build_structure) on graphs handed over
// from Python: no GPU is touched, so it runs in the build container.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/micro/lba_host_time.hip \
//            -Iinclude -Lorb_slam3_comments_ghr_amd -lorbslam3_amd -o tools/micro/liblba_host_time.so
#define OSG_LBA_STRUCT_PROF
#ifdef LBA_HOST_BA_SRC
#include LBA_HOST_BA_SRC
#else
#include "../../orb_slam3_comments_ghr_amd/csrc/ba.hip"
#endif

extern "C" double lba_host_time_ms(const osg_ba_graph *G, int reps, int *ncontrib)
{
    osg_ctx ctx;
    LbaHost H;
    double best = 1e30;
    for (int r = 0; r < reps; r++) {
        H.reset();
        const auto t0 = std::chrono::steady_clock::now();
        if (build_structure(&ctx, G, H) != OSG_OK) return -1;
        best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    *ncontrib = H.pair_start.empty() ? 0 : H.pair_start.back();
    return best;
}

// FNV-1a over every structure array of the last build (identity check across rewrites)
extern "C" unsigned long long lba_host_struct_hash(const osg_ba_graph *G)
{
    osg_ctx ctx;
    LbaHost H;
    if (build_structure(&ctx, G, H) != OSG_OK) return 0;
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const std::vector<int32_t> &v) {
        const unsigned char *p = (const unsigned char *)v.data();
        for (size_t i = 0; i < v.size() * 4; i++) h = (h ^ p[i]) * 1099511628211ull;
        h = (h ^ v.size()) * 1099511628211ull;
    };
    // the contributions' second blocks (pair_b; pair_ab's odd entries in older builds)
#ifdef LBA_HOST_PAIR_AB
    std::vector<int32_t> pb(std::max<size_t>(H.pair_ab.size() / 2, 1));
    for (size_t k = 0; k < H.pair_ab.size() / 2; k++) pb[k] = H.pair_ab[2 * k + 1];
#else
    std::vector<int32_t> &pb = H.pair_b;
#endif
    for (auto *v : {&H.blk_first, &H.blk_last, &H.col_rows_start, &H.col_rows, &H.live_pairs, &H.pose_h, &H.hp_pose,
                    &H.point_h, &H.hl_point, &H.lm_e_start, &H.lm_e, &H.lg_start, &H.lm_b_start, &H.blk_pose,
                    &H.edge_blk, &H.blk_lm, &H.hp_e_start, &H.hp_e, &H.hp_b_start, &H.hp_b, &H.pair_start,
                    &pb, &H.chunk_start, &H.pair_chunk, &H.pair_rank, &H.rs_pose, &H.rs_rank0,
                    &H.rs_chunk_start, &H.rs_chunk, &H.hp_rs_start, &H.rs_order, &H.rs_cdesc, &H.rs_info, &H.hp_b_lm,
                    &H.live_chunk, &H.env_off})
        mix(*v);
    const int sc[] = {H.np, H.npt, H.ne, H.nhp, H.nhl, H.nblk, H.npairs, H.nchunks, H.ge, H.gl, H.gll, H.gu,
                      H.nblk_red, H.npart, H.n_rs, H.max_col_rows, (int)H.multi};
    for (int v : sc) h = (h ^ (unsigned)v) * 1099511628211ull;
    return h;
}

extern "C" void lba_host_time_phases(double *out16)
{
    for (int k = 0; k < 16; k++) {
        out16[k] = g_struct_cp[k];
        g_struct_cp[k] = 0;
    }
}

// osg_parallel_for under concurrent callers: T threads, each running `loops` loops of n indices that
// sum i * i; returns the number of wrong sums (0 expected)
extern "C" int pool_stress(int T, int loops, int n)
{
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            for (int k = 0; k < loops; k++) {
                std::vector<long long> v(n, 0);
                osg_parallel_for(n, 1 + (t + k) % 16, [&](int i) { v[i] = (long long)i * i; });
                long long s = 0;
                for (int i = 0; i < n; i++) s += v[i];
                const long long want = (long long)(n - 1) * n * (2LL * n - 1) / 6;
                if (s != want) bad++;
            }
        });
    for (auto &x : th) x.join();
    return bad.load();
}

// the reduced system's size and envelope reach of the last structure build: {n, blocks, max rows below a
// column block inside the envelope}
extern "C" void lba_host_envelope(const osg_ba_graph *G, int *out3)
{
    osg_ctx ctx;
    LbaHost H;
    out3[0] = out3[1] = out3[2] = -1;
    if (build_structure(&ctx, G, H) != OSG_OK) return;
    out3[0] = 6 * H.nhp;
    out3[1] = H.nblk_red;
    out3[2] = H.max_col_rows;
}
