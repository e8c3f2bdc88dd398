// adapter_driver.cpp — runs adapters/orbslam3/osg_orbslam3.h on mock ORB-SLAM3 objects built from
// arrays written by tests/test_adapter.py, and writes the adapter's results back (test-only).
//
//   adapter_driver MODE in.arrays out.arrays      MODE: mps last kf bow_kf_f bow_kf_kf pose lba fuse fuse_sim3 triang distinct sim3 sim3_kfs sim3pair init stereo fisheye gba merge_lba orb
//                                                       bow, and the batched forms bow_kf_f_batch pose_batch last_batch mps_batch
//                                                       stereo_batch bow_batch
#include <deque>

#include "driver_common.h"

// Batched forms ("<mode>_batch"): "batch.n" problems under the prefixes "b0.", "b1.", ... with the
// single mode's arrays and the same "params"; outputs concatenated in problem order.
static void run_batch_mode(const std::string &mode, const Arrays &in, const float *prm, Arrays &out)
{
    namespace oa = osg_orbslam3;
    const int B = get(in, "batch.n").p<int32_t>()[0];
    std::vector<std::unique_ptr<MapPoint>> pool;
    std::vector<int32_t> nm(B, -7);
    auto pre = [](int b) { return "b" + std::to_string(b) + "."; };
    if (mode == "bow_kf_f_batch") {
        std::deque<KeyFrame> K(B);
        std::deque<Frame> F(B);
        std::vector<KeyFrame *> kp;
        std::vector<Frame *> fp;
        for (int b = 0; b < B; b++) {
            build_bow_kf_f_problem(in, pre(b), K[b], F[b], pool);
            kp.push_back(&K[b]);
            fp.push_back(&F[b]);
        }
        std::vector<std::vector<MapPoint *>> matches;
        oa::search_by_bow_kf_f_batch<MockHooks>(kp, fp, matches, prm[0], prm[1] != 0, nm.data());
        std::vector<int32_t> all;
        for (auto &m : matches) for (int32_t v : slot_ids(m)) all.push_back(v);
        out["out_mp"] = make('i', all);
    } else if (mode == "pose_batch") {
        std::deque<Frame> F(B);
        std::deque<Camera> c(B), c2(B);
        std::vector<Frame *> fp;
        for (int b = 0; b < B; b++) {
            build_pose_problem(in, pre(b), F[b], c[b], c2[b], pool);
            fp.push_back(&F[b]);
        }
        oa::pose_optimization_batch<MockHooks>(fp, nm.data());
        std::vector<double> poses;
        std::vector<uint8_t> outl;
        for (int b = 0; b < B; b++) {
            poses.insert(poses.end(), F[b].pose, F[b].pose + 7);
            for (int i = 0; i < F[b].N; i++) outl.push_back(F[b].mvbOutlier[i]);
        }
        out["pose"] = make('d', poses);
        out["outlier"] = make('b', outl);
    } else if (mode == "last_batch") {
        std::deque<Frame> CF(B), LF(B);
        std::vector<Frame *> cp;
        std::vector<const Frame *> lp;
        for (int b = 0; b < B; b++) {
            build_last_problem(in, pre(b), CF[b], LF[b], pool);
            CF[b].tlc_z_value = prm[3];
            cp.push_back(&CF[b]);
            lp.push_back(&LF[b]);
        }
        oa::search_by_projection_last_batch<MockHooks>(cp, lp, prm[0], prm[1] != 0, prm[2] != 0, nm.data());
        std::vector<int32_t> all;
        for (int b = 0; b < B; b++) for (int32_t v : slot_ids(CF[b].mvpMapPoints)) all.push_back(v);
        out["slot_mp"] = make('i', all);
    } else if (mode == "mps_batch") {
        std::deque<Frame> F(B);
        std::deque<std::vector<MapPoint *>> Q(B);
        std::vector<Frame *> fp;
        std::vector<const std::vector<MapPoint *> *> qp;
        for (int b = 0; b < B; b++) {
            build_mps_problem(in, pre(b), F[b], Q[b], pool);
            fp.push_back(&F[b]);
            qp.push_back(&Q[b]);
        }
        oa::search_by_projection_mps_batch<MockHooks>(fp, qp, prm[1], prm[2] != 0, prm[3], prm[0], nm.data());
        std::vector<int32_t> all;
        for (int b = 0; b < B; b++) for (int32_t v : slot_ids(F[b].mvpMapPoints)) all.push_back(v);
        out["slot_mp"] = make('i', all);
    } else if (mode == "stereo_batch") {
        std::deque<Frame> F(B);
        std::deque<ORBextractor> el(B), er(B);
        std::vector<Frame *> fp;
        for (int b = 0; b < B; b++) {
            build_stereo_problem(in, pre(b), F[b], el[b], er[b]);
            fp.push_back(&F[b]);
        }
        oa::compute_stereo_matches_batch(fp, nm.data());
        std::vector<float> ur, depth;
        for (int b = 0; b < B; b++) {
            ur.insert(ur.end(), F[b].mvuRight.begin(), F[b].mvuRight.end());
            depth.insert(depth.end(), F[b].mvDepth.begin(), F[b].mvDepth.end());
        }
        out["ur"] = make('f', ur);
        out["depth"] = make('f', depth);
    } else if (mode == "bow_batch") {  // ComputeBoW, B frames in one launch
        osg_vocabulary *voc = build_vocabulary(in);
        std::deque<Frame> F(B);
        std::vector<Frame *> fp;
        for (int b = 0; b < B; b++) {
            build_bow_frame(in, pre(b), F[b]);
            fp.push_back(&F[b]);
        }
        oa::compute_bow_batch(fp, voc);
        osg_vocabulary_destroy(voc);
        std::vector<int32_t> word, nid, ns, feat, counts;
        std::vector<double> value;
        for (int b = 0; b < B; b++) append_bow(F[b], word, value, nid, ns, feat, counts);
        out["word"] = make('i', word);
        out["value"] = make('d', value);
        out["node_id"] = make('i', nid);
        out["node_start"] = make('i', ns);
        out["feat"] = make('i', feat);
        out["counts"] = make('i', counts);
    } else {
        throw std::runtime_error("unknown batch mode " + mode);
    }
    out["nmatches"] = make('i', nm);
}

int main(int argc, char **argv)
{
    if (argc != 4) {
        fprintf(stderr, "usage: %s MODE in out\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    try {
        const Arrays in = read_arrays(argv[2]);
        Arrays out;
        std::vector<std::unique_ptr<MapPoint>> pool;
        const float *prm = has(in, "params") ? get(in, "params").p<float>() : nullptr;
        if (mode == "mps") {
            Frame F;
            std::vector<MapPoint *> q;
            build_mps_problem(in, "", F, q, pool);
            // params: nnratio th far thfar
            const int nm = osg_orbslam3::search_by_projection_mps<MockHooks>(F, q, prm[1], prm[2] != 0, prm[3], prm[0]);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["slot_mp"] = make('i', slot_ids(F.mvpMapPoints));
        } else if (mode == "last") {
            Frame CF, LF;
            build_last_problem(in, "", CF, LF, pool);
            CF.tlc_z_value = prm[3];
            // params: th mono ori tlc_z
            const int nm = osg_orbslam3::search_by_projection_last<MockHooks>(CF, LF, prm[0], prm[1] != 0, prm[2] != 0);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["slot_mp"] = make('i', slot_ids(CF.mvpMapPoints));
        } else if (mode == "kf") {
            Frame CF;
            build_frame(in, CF);
            build_slots(in, "", CF, pool);
            KeyFrame K;
            const int n = (int)get(in, "K.mp_id").n;
            K.N = n;
            K.mvKeysUn.resize(n);
            K.mvpMapPoints.assign(n, nullptr);
            for (int i = 0; i < n; i++) {
                K.mvKeysUn[i].angle = get(in, "K.angle").p<float>()[i];
                pool.emplace_back(new MapPoint());
                MapPoint *p = pool.back().get();
                p->mnId = (unsigned long)get(in, "K.mp_id").p<int32_t>()[i];
                std::memcpy(p->desc.buf.data(), get(in, "K.desc").p<uint8_t>() + 32 * i, 32);
                p->proj_ok = get(in, "K.valid").p<uint8_t>()[i];
                p->proj_u = get(in, "K.u").p<float>()[i];
                p->proj_v = get(in, "K.v").p<float>()[i];
                p->proj_level = get(in, "K.pred_level").p<int32_t>()[i];
                K.mvpMapPoints[i] = p;
            }
            std::set<MapPoint *> already;
            // params: th orbdist ori
            const int nm = osg_orbslam3::search_by_projection_kf<MockHooks>(CF, &K, already, prm[0], (int)prm[1], prm[2] != 0);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["slot_mp"] = make('i', slot_ids(CF.mvpMapPoints));
        } else if (mode == "bow_kf_f") {
            KeyFrame K;
            Frame F;
            build_bow_kf_f_problem(in, "", K, F, pool);
            std::vector<MapPoint *> matches;
            // params: nnratio ori
            const int nm = osg_orbslam3::search_by_bow_kf_f<MockHooks>(&K, F, matches, prm[0], prm[1] != 0);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["out_mp"] = make('i', slot_ids(matches));
        } else if (mode == "bow_kf_kf") {
            KeyFrame K1, K2;
            build_bow_kf(in, "B1.", K1, pool);
            build_bow_kf(in, "B2.", K2, pool);
            std::vector<MapPoint *> matches;
            const int nm = osg_orbslam3::search_by_bow_kf_kf<MockHooks>(&K1, &K2, matches, prm[0], prm[1] != 0);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["out_mp"] = make('i', slot_ids(matches));
        } else if (mode == "pose") {
            Frame F;
            Camera c, c2;
            build_pose_problem(in, "", F, c, c2, pool);
            const int n = F.N;
            ProbeMutex probe;  // params[0] != 0: pass a MapPoint::mGlobalMutex stand-in and report its use
            const bool use_probe = prm && prm[0] != 0;
            if (use_probe) g_probe = &probe;
            const int inl = use_probe ? osg_orbslam3::pose_optimization<MockHooks>(&F, &probe)
                                      : osg_orbslam3::pose_optimization<MockHooks>(&F);
            g_probe = nullptr;
            out["lock_stats"] = make('i', std::vector<int32_t>{probe.locks, g_gather_unlocked, g_apply_locked,
                                                               g_apply_try_lock_failed, (int32_t)probe.held});
            std::vector<uint8_t> outl(n);
            for (int i = 0; i < n; i++) outl[i] = F.mvbOutlier[i];
            out["n_inliers"] = make('i', std::vector<int32_t>{inl});
            out["pose"] = make('d', std::vector<double>(F.pose, F.pose + 7));
            out["outlier"] = make('b', outl);
        } else if (mode == "lba") {
            const int np = (int)(get(in, "G.pose").n / 7), npt = (int)(get(in, "G.point").n / 3), ne = (int)get(in, "G.e_pose").n;
            Camera c;
            Map map;
            std::vector<KeyFrame> kf;
            std::vector<MapPoint> mp;
            build_ba_world(in, map, c, kf, mp);
            std::list<KeyFrame *> local, fixedc;
            const uint8_t *fx = get(in, "G.pose_fixed").p<uint8_t>();
            for (int i = 0; i < np; i++) (fx[i] ? fixedc : local).push_back(&kf[i]);
            std::list<MapPoint *> mps;
            for (auto &p : mp) mps.push_back(&p);
            bool stop = false;
            // optional: params[0] = the map's init KeyFrame id (default none); "G.mp_bad" = MapPoints
            // another thread marks bad while the solve runs (in the graph, skipped at classification)
            const unsigned long init_id = prm ? (unsigned long)prm[0] : ~0ul;
            if (has(in, "G.mp_bad"))
                for (int j = 0; j < npt; j++) mp[j].bad = get(in, "G.mp_bad").p<uint8_t>()[j] != 0;
            auto o = osg_orbslam3::local_bundle_adjustment<MockHooks>(local, fixedc, mps, &map, init_id, &stop, false);
            std::vector<uint8_t> bad(ne, 0);
            std::vector<int32_t> erased;
            {
                std::map<std::pair<KeyFrame *, MapPoint *>, int> edge_of;
                for (int e = 0; e < ne; e++)
                    edge_of[{&kf[get(in, "G.e_pose").p<int32_t>()[e]], &mp[get(in, "G.e_point").p<int32_t>()[e]]}] = e;
                for (auto &km : o.to_erase) {
                    bad[edge_of[km]] = 1;
                    erased.push_back(edge_of[km]);
                }
            }
            out["erased"] = make('i', erased);
            out["counts"] = make('i', std::vector<int32_t>{o.num_fixedKF, o.num_OptKF, o.num_MPs, o.num_edges});
            osg_orbslam3::apply_local_bundle_adjustment<MockHooks>(o);
            std::vector<double> pose(7 * (size_t)np), point(3 * (size_t)npt);
            for (int i = 0; i < np; i++) std::memcpy(&pose[7 * i], kf[i].pose, 56);
            for (int j = 0; j < npt; j++) std::memcpy(&point[3 * j], mp[j].pos, 24);
            out["pose"] = make('d', pose);
            out["point"] = make('d', point);
            out["edge_bad"] = make('b', bad);
            out["num_edges"] = make('i', std::vector<int32_t>{o.num_edges});
        } else if (mode == "merge_lba") {
            // the "lba" arrays; params: n_fixed stop.  vpFixedKF = KeyFrames [0, n_fixed), vpAdjustKF the
            // rest, pMainKF the last; out: poses, points, the erased (KeyFrame, MapPoint) pairs in order
            const int np = (int)(get(in, "G.pose").n / 7), npt = (int)(get(in, "G.point").n / 3);
            Camera c;
            Map map;
            std::vector<KeyFrame> kf;
            std::vector<MapPoint> mp;
            build_ba_world(in, map, c, kf, mp);
            std::vector<KeyFrame *> fixedk, adjust;
            for (int i = 0; i < np; i++) (i < (int)prm[0] ? fixedk : adjust).push_back(&kf[i]);
            bool stop = prm[1] != 0;
            auto o = osg_orbslam3::merge_local_bundle_adjustment<MockHooks, KeyFrame, MapPoint>(&kf[np - 1], adjust,
                                                                                             fixedk, &stop);
            std::vector<int32_t> erased;
            for (auto &km : o.to_erase) {
                erased.push_back((int32_t)(km.first - kf.data()));
                erased.push_back((int32_t)(km.second - mp.data()));
            }
            if (!o.aborted) osg_orbslam3::apply_merge_local_bundle_adjustment<MockHooks>(o);
            std::vector<double> pose(7 * (size_t)np), point(3 * (size_t)npt);
            for (int i = 0; i < np; i++) std::memcpy(&pose[7 * i], kf[i].pose, 56);
            for (int j = 0; j < npt; j++) std::memcpy(&point[3 * j], mp[j].pos, 24);
            out["pose"] = make('d', pose);
            out["point"] = make('d', point);
            out["erased"] = make('i', erased);
            out["aborted"] = make('i', std::vector<int32_t>{(int32_t)o.aborted});
        } else if (mode == "gba") {
            // the "lba" arrays; params: nIterations bRobust nLoopKF.  KeyFrame 0 is the map's init and
            // origin KeyFrame: nLoopKF 0 writes into the map, anything else into mTcwGBA / mPosGBA
            const int np = (int)(get(in, "G.pose").n / 7), npt = (int)(get(in, "G.point").n / 3);
            Camera c;
            Map map;
            std::vector<KeyFrame> kf;
            std::vector<MapPoint> mp;
            build_ba_world(in, map, c, kf, mp);
            std::vector<KeyFrame *> vk;
            std::vector<MapPoint *> vm;
            for (auto &k : kf) vk.push_back(&k);
            for (auto &p : mp) vm.push_back(&p);
            bool stop = false;
            const unsigned long nLoop = (unsigned long)prm[2];
            auto o = osg_orbslam3::bundle_adjustment<MockHooks>(vk, vm, 0ul, (int)prm[0], &stop, prm[1] != 0);
            osg_orbslam3::apply_bundle_adjustment<MockHooks>(o, nLoop, nLoop == 0);
            std::vector<double> pose(7 * (size_t)np), point(3 * (size_t)npt), pose_gba(7 * (size_t)np),
                point_gba(3 * (size_t)npt);
            std::vector<int32_t> ba_for;
            for (int i = 0; i < np; i++) {
                std::memcpy(&pose[7 * i], kf[i].pose, 56);
                std::memcpy(&pose_gba[7 * i], kf[i].pose_gba, 56);
                ba_for.push_back((int32_t)kf[i].mnBAGlobalForKF);
            }
            for (int j = 0; j < npt; j++) {
                std::memcpy(&point[3 * j], mp[j].pos, 24);
                std::memcpy(&point_gba[3 * j], mp[j].pos_gba, 24);
                ba_for.push_back((int32_t)mp[j].mnBAGlobalForKF);
            }
            out["pose"] = make('d', pose);
            out["point"] = make('d', point);
            out["pose_gba"] = make('d', pose_gba);
            out["point_gba"] = make('d', point_gba);
            out["ba_for"] = make('i', ba_for);
            out["iterations"] = make('i', std::vector<int32_t>{o.iterations});
        } else if (mode == "fuse" || mode == "fuse_sim3") {
            // pool of MapPoints "P.*" (index = id), the keyframe's slot occupants "K.slot_mp", the
            // list to fuse "L.list" (pool indices, -1 = NULL); params: th right
            KeyFrame K;
            build_kf_frame(in, K);
            const Arr &is2 = get(in, "K.inv_s2");
            K.mvInvLevelSigma2.assign(is2.p<float>(), is2.p<float>() + is2.n);
            const int np = (int)get(in, "P.nobs").n;
            std::vector<MapPoint> P(np);
            for (int i = 0; i < np; i++) {
                MapPoint &p = P[i];
                p.mnId = (unsigned long)i;
                std::memcpy(p.desc.buf.data(), get(in, "P.desc").p<uint8_t>() + 32 * i, 32);
                p.proj_ok = get(in, "P.ok").p<uint8_t>()[i];
                p.proj_u = get(in, "P.u").p<float>()[i];
                p.proj_v = get(in, "P.v").p<float>()[i];
                p.proj_fuse_ur = get(in, "P.ur").p<float>()[i];
                p.proj_level = get(in, "P.level").p<int32_t>()[i];
                p.bad = get(in, "P.bad").p<uint8_t>()[i];
                p.nobs = get(in, "P.nobs").p<int32_t>()[i];
            }
            const int32_t *sm = get(in, "K.slot_mp").p<int32_t>();
            for (int k = 0; k < K.N; k++)
                if (sm[k] >= 0) {
                    K.mvpMapPoints[k] = &P[sm[k]];
                    P[sm[k]].obs[&K] = std::make_tuple(k, -1);
                }
            const Arr &L = get(in, "L.list");
            std::vector<MapPoint *> list(L.n);
            for (size_t i = 0; i < L.n; i++) list[i] = L.p<int32_t>()[i] < 0 ? nullptr : &P[L.p<int32_t>()[i]];
            int nf;
            std::vector<int32_t> repl(L.n, -1);
            if (mode == "fuse") {
                nf = osg_orbslam3::fuse<MockHooks>(&K, list, prm[0], prm[1] != 0);
            } else {
                std::vector<MapPoint *> vpReplace(L.n, nullptr);
                nf = osg_orbslam3::fuse_sim3<MockHooks>(&K, Sim3{}, list, prm[0], vpReplace);
                for (size_t i = 0; i < L.n; i++) repl[i] = vpReplace[i] ? (int32_t)vpReplace[i]->mnId : -1;
            }
            std::vector<uint8_t> bad(np);
            std::vector<int32_t> nobs(np);
            for (int i = 0; i < np; i++) {
                bad[i] = P[i].bad;
                nobs[i] = P[i].nobs;
            }
            out["nfused"] = make('i', std::vector<int32_t>{nf});
            out["slot_mp"] = make('i', slot_ids(K.mvpMapPoints));
            out["bad"] = make('b', bad);
            out["nobs"] = make('i', nobs);
            out["replace"] = make('i', repl);
        } else if (mode == "triang") {
            // keyframes "A." / "B.", geometry "G.geom" {ep_x, ep_y, F12[36], pinhole}; params: only_stereo coarse ori
            KeyFrame A, B;
            build_triang_kf(in, "A.", A, pool);
            build_triang_kf(in, "B.", B, pool);
            const float *g = get(in, "G.geom").p<float>();
            A.triang_geom.ep_x = g[0];
            A.triang_geom.ep_y = g[1];
            std::memcpy(A.triang_geom.F12, g + 2, sizeof(float) * 36);
            A.triang_geom.pinhole = g[38] != 0;
            if (has(in, "G.kb8")) {  // KannalaBrandt8: R12[36] t12[12] kb[32]
                const float *k = get(in, "G.kb8").p<float>();
                std::memcpy(A.triang_geom.R12, k, sizeof(float) * 36);
                std::memcpy(A.triang_geom.t12, k + 36, sizeof(float) * 12);
                std::memcpy(A.triang_geom.kb, k + 48, sizeof(float) * 32);
            }
            std::vector<std::pair<size_t, size_t>> pairs;
            const int nm = osg_orbslam3::search_for_triangulation<MockHooks>(&A, &B, pairs, prm[0] != 0, prm[1] != 0,
                                                                              prm[2] != 0);
            std::vector<int32_t> flat;
            for (auto &pr : pairs) {
                flat.push_back((int32_t)pr.first);
                flat.push_back((int32_t)pr.second);
            }
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["pairs"] = make('i', flat);
        } else if (mode == "sim3" || mode == "sim3_kfs") {
            // keyframe "F.*"; MapPoint pool "P.*" (desc ok u v level bad); "L.list" pool indices;
            // "V.matched" initial vpMatched (pool index, -1); params: th ratio
            KeyFrame K;
            build_kf_frame(in, K);
            const int np = (int)get(in, "P.bad").n;
            std::vector<MapPoint> P(np);
            for (int i = 0; i < np; i++) {
                MapPoint &p = P[i];
                p.mnId = (unsigned long)i;
                std::memcpy(p.desc.buf.data(), get(in, "P.desc").p<uint8_t>() + 32 * i, 32);
                p.proj_ok = get(in, "P.ok").p<uint8_t>()[i];
                p.proj_u = get(in, "P.u").p<float>()[i];
                p.proj_v = get(in, "P.v").p<float>()[i];
                p.proj_level = get(in, "P.level").p<int32_t>()[i];
                p.bad = get(in, "P.bad").p<uint8_t>()[i];
            }
            const Arr &L = get(in, "L.list");
            std::vector<MapPoint *> list(L.n);
            std::vector<KeyFrame> owners(7);
            std::vector<KeyFrame *> list_kfs(L.n);
            for (size_t i = 0; i < L.n; i++) {
                list[i] = &P[L.p<int32_t>()[i]];
                list_kfs[i] = &owners[i % 7];
            }
            std::vector<MapPoint *> matched(K.N, nullptr);
            std::vector<KeyFrame *> matched_kf(K.N, nullptr);
            for (int k = 0; k < K.N; k++) {
                const int32_t m = get(in, "V.matched").p<int32_t>()[k];
                if (m >= 0) matched[k] = &P[m];
            }
            int nm;
            if (mode == "sim3")
                nm = osg_orbslam3::search_by_projection_sim3<MockHooks, KeyFrame>(&K, Sim3{}, list, nullptr, matched,
                                                                                 nullptr, (int)prm[0], prm[1]);
            else
                nm = osg_orbslam3::search_by_projection_sim3<MockHooks, KeyFrame>(&K, Sim3{}, list, &list_kfs, matched,
                                                                                 &matched_kf, (int)prm[0], prm[1]);
            std::vector<int32_t> mo(K.N, -1), mk(K.N, -1);
            for (int k = 0; k < K.N; k++) {
                if (matched[k]) mo[k] = (int32_t)matched[k]->mnId;
                if (matched_kf[k]) mk[k] = (int32_t)(matched_kf[k] - owners.data());
            }
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["matched"] = make('i', mo);
            out["matched_kf"] = make('i', mk);
        } else if (mode == "sim3pair") {
            // SearchBySim3: keyframes "F.*" (KF1) and "G.*" (KF2); per KF1 slot "A.*" (has desc ok u v level
            // bad) of its MapPoint projected into KF2, per KF2 slot "B.*" likewise into KF1; "V.matched":
            // initial vpMatches12 as KF2 slot indices (-1); params: th.  out: matched (KF2 slot or -1)
            KeyFrame K1, K2;
            build_kf_frame(in, K1);
            {
                Arrays g;
                for (auto &kv : in)
                    if (kv.first.rfind("G.", 0) == 0) g["F." + kv.first.substr(2)] = kv.second;
                build_kf_frame(g, K2);
            }
            std::vector<MapPoint> P1(K1.N), P2(K2.N);
            auto fill = [&](const char *pre, std::vector<MapPoint> &P, KeyFrame &K, KeyFrame &other, int d) {
                const std::string a(pre);
                for (int i = 0; i < K.N; i++) {
                    MapPoint &p = P[i];
                    if (!get(in, a + "has").p<uint8_t>()[i]) continue;
                    std::memcpy(p.desc.buf.data(), get(in, a + "desc").p<uint8_t>() + 32 * i, 32);
                    p.s3_ok[d] = get(in, a + "ok").p<uint8_t>()[i];
                    p.s3_u[d] = get(in, a + "u").p<float>()[i];
                    p.s3_v[d] = get(in, a + "v").p<float>()[i];
                    p.s3_level[d] = get(in, a + "level").p<int32_t>()[i];
                    p.bad = get(in, a + "bad").p<uint8_t>()[i];
                    p.obs[&K] = std::make_tuple(i, -1);
                    K.mvpMapPoints[i] = &p;
                }
                (void)other;
            };
            fill("A.", P1, K1, K2, 0);
            fill("B.", P2, K2, K1, 1);
            std::vector<MapPoint *> m12(K1.N, nullptr);
            for (int i = 0; i < K1.N; i++) {
                const int32_t j = get(in, "V.matched").p<int32_t>()[i];
                if (j >= 0) {
                    m12[i] = &P2[j];
                    P2[j].obs[&K2] = std::make_tuple(j, -1);
                }
            }
            const int nm = osg_orbslam3::search_by_sim3<MockHooks, KeyFrame>(&K1, &K2, m12, Sim3{}, prm[0]);
            std::vector<int32_t> mo(K1.N, -1);
            for (int i = 0; i < K1.N; i++)
                if (m12[i]) mo[i] = (int32_t)(m12[i] - P2.data());
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["matched"] = make('i', mo);
        } else if (mode == "init") {
            // F1 "F.*", F2 "G.*", vbPrevMatched "V.prev" (n1 x 2); params: windowSize nnratio checkOri
            Frame F1, F2;
            build_frame(in, F1, "F.");
            build_frame(in, F2, "G.");
            const Arr &pv = get(in, "V.prev");
            std::vector<cv::Point2f> prev(F1.N);
            for (int i = 0; i < F1.N; i++) {
                prev[i].x = pv.p<float>()[2 * i];
                prev[i].y = pv.p<float>()[2 * i + 1];
            }
            std::vector<int> m12;
            const int nm = osg_orbslam3::search_for_initialization<MockHooks>(F1, F2, prev, m12, (int)prm[0], prm[1],
                                                                               prm[2] != 0);
            std::vector<float> po(2 * (size_t)F1.N);
            for (int i = 0; i < F1.N; i++) {
                po[2 * i] = prev[i].x;
                po[2 * i + 1] = prev[i].y;
            }
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["m12"] = make('i', std::vector<int32_t>(m12.begin(), m12.end()));
            out["prev"] = make('f', po);
        } else if (mode == "bow") {  // Frame::ComputeBoW, twice: the second call keeps mBowVec (not empty)
            osg_vocabulary *voc = build_vocabulary(in);
            Frame F;
            build_bow_frame(in, "", F);
            osg_orbslam3::compute_bow(F, voc);
            std::vector<int32_t> word, nid, ns, feat, counts;
            std::vector<double> value;
            append_bow(F, word, value, nid, ns, feat, counts);
            const auto bow = F.mBowVec;
            F.mFeatVec.clear();
            osg_orbslam3::compute_bow(F, voc);
            osg_vocabulary_destroy(voc);
            out["word"] = make('i', word);
            out["value"] = make('d', value);
            out["node_id"] = make('i', nid);
            out["node_start"] = make('i', ns);
            out["feat"] = make('i', feat);
            out["counts"] = make('i', counts);
            out["second_call_kept"] = make('i', std::vector<int32_t>{F.mBowVec == bow && F.mFeatVec.empty() ? 1 : 0});
        } else if (mode == "stereo") {
            Frame F;
            ORBextractor el, er;
            build_stereo_problem(in, "", F, el, er);
            F.mvuRight.assign(F.N, 123.0f);  // overwritten, as the reference's are
            const int nm = osg_orbslam3::compute_stereo_matches(F);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["ur"] = make('f', F.mvuRight);
            out["depth"] = make('f', F.mvDepth);
        } else if (mode.size() > 6 && mode.compare(mode.size() - 6, 6, "_batch") == 0) {
            run_batch_mode(mode, in, prm, out);
        } else if (mode == "fisheye") {
            // "FE.kl" / "FE.kr" (x, y), "FE.ol" / "FE.or", "FE.dl" / "FE.dr", "FE.mono" (monoLeft, monoRight),
            // "FE.sig2", "FE.cam" (2 x 8 KannalaBrandt8), "FE.R" (3x3), "FE.t"
            Frame F;
            const int nl = (int)get(in, "FE.ol").n, nr = (int)get(in, "FE.or").n;
            auto kps = [&](const char *k, const char *o, int cnt) {
                std::vector<cv::KeyPoint> v(cnt);
                for (int i = 0; i < cnt; i++) {
                    v[i].pt.x = get(in, k).p<float>()[2 * i];
                    v[i].pt.y = get(in, k).p<float>()[2 * i + 1];
                    v[i].octave = get(in, o).p<int32_t>()[i];
                }
                return v;
            };
            F.N = nl + nr;
            F.Nleft = nl;
            F.Nright = nr;
            F.mvKeys = kps("FE.kl", "FE.ol", nl);
            F.mvKeysRight = kps("FE.kr", "FE.or", nr);
            F.mDescriptors = cv::Mat(nl, 32);
            std::memcpy(F.mDescriptors.buf.data(), get(in, "FE.dl").b.data(), (size_t)nl * 32);
            F.mDescriptorsRight = cv::Mat(nr, 32);
            std::memcpy(F.mDescriptorsRight.buf.data(), get(in, "FE.dr").b.data(), (size_t)nr * 32);
            F.monoLeft = get(in, "FE.mono").p<int32_t>()[0];
            F.monoRight = get(in, "FE.mono").p<int32_t>()[1];
            const Arr &s2 = get(in, "FE.sig2");
            F.mvLevelSigma2.assign(s2.p<float>(), s2.p<float>() + s2.n);
            Camera c1, c2;
            c1.type = c2.type = OSG_CAM_KB8;
            c1.params.assign(get(in, "FE.cam").p<float>(), get(in, "FE.cam").p<float>() + 8);
            c2.params.assign(get(in, "FE.cam").p<float>() + 8, get(in, "FE.cam").p<float>() + 16);
            F.mpCamera = &c1;
            F.mpCamera2 = &c2;
            for (int k = 0; k < 9; k++) F.mRlr.a[k] = get(in, "FE.R").p<float>()[k];
            for (int k = 0; k < 3; k++) F.mtlr.a[k] = get(in, "FE.t").p<float>()[k];
            const int nm = osg_orbslam3::compute_stereo_fisheye_matches(F);
            std::vector<float> p3d(3 * (size_t)nl, 0.f);
            for (int i = 0; i < nl; i++)
                if (F.mvLeftToRightMatch[i] >= 0)
                    for (int k = 0; k < 3; k++) p3d[3 * (size_t)i + k] = F.mvStereo3Dpoints[i](k);
            out["nmatches"] = make('i', std::vector<int32_t>{nm, F.mnCloseMPs});
            out["l2r"] = make('i', std::vector<int32_t>(F.mvLeftToRightMatch.begin(), F.mvLeftToRightMatch.end()));
            out["r2l"] = make('i', std::vector<int32_t>(F.mvRightToLeftMatch.begin(), F.mvRightToLeftMatch.end()));
            out["depth"] = make('f', F.mvDepth);
            out["ur"] = make('f', F.mvuRight);
            out["p3d"] = make('f', p3d);
        } else if (mode == "orb") {
            // levels "O.raw" / "O.blur" concatenated with "O.dims" (rows, cols); keypoints "O.x", "O.y",
            // "O.level" (sorted by level); "O.pattern" (512 x 2), "O.umax" (16).  mvImagePyramid levels are
            // ROIs of wider rows (step = cols + 7); the blurred levels are continuous clones
            const Arr &dims = get(in, "O.dims");
            const int levels = (int)dims.n / 2;
            ORBextractor ex;
            std::vector<cv::Mat> blurred;
            const uint8_t *sr = get(in, "O.raw").p<uint8_t>(), *sb = get(in, "O.blur").p<uint8_t>();
            for (int l = 0; l < levels; l++) {
                const int rows = dims.p<int32_t>()[2 * l], cols = dims.p<int32_t>()[2 * l + 1];
                cv::Mat m(rows, cols, (size_t)cols + 7), b(rows, cols);
                for (int r = 0; r < rows; r++) std::memcpy(m.ptr<unsigned char>(r), sr + (size_t)r * cols, cols);
                std::memcpy(b.buf.data(), sb, (size_t)rows * cols);
                sr += (size_t)rows * cols;
                sb += (size_t)rows * cols;
                ex.mvImagePyramid.push_back(std::move(m));
                blurred.push_back(std::move(b));
            }
            const Arr &pa = get(in, "O.pattern"), &um = get(in, "O.umax");
            for (size_t i = 0; i < pa.n / 2; i++) ex.pattern.push_back(cv::Point{pa.p<int32_t>()[2 * i], pa.p<int32_t>()[2 * i + 1]});
            ex.umax.assign(um.p<int32_t>(), um.p<int32_t>() + um.n);
            std::vector<std::vector<cv::KeyPoint>> all(levels);
            const Arr &kx = get(in, "O.x");
            for (size_t i = 0; i < kx.n; i++) {
                cv::KeyPoint kp;
                kp.pt.x = kx.p<float>()[i];
                kp.pt.y = get(in, "O.y").p<float>()[i];
                kp.angle = -7.0f;  // overwritten
                all[get(in, "O.level").p<int32_t>()[i]].push_back(kp);
            }
            std::vector<uint8_t> desc;
            const int n_out = osg_orbslam3::orb_describe(ex.mvImagePyramid, blurred, all, ex.pattern, ex.umax, desc);
            std::vector<float> ang;
            for (auto &lv : all)
                for (auto &kp : lv) ang.push_back(kp.angle);
            out["n_out"] = make('i', std::vector<int32_t>{n_out});
            out["angle"] = make('f', ang);
            out["desc"] = make('b', desc);
        } else if (mode == "detect") {
            // levels "D.raw" concatenated with "D.dims" (rows, cols), stored as ROIs (step = cols + 5);
            // "D.nf" mnFeaturesPerLevel, "D.scale" mvScaleFactor, "D.th" (iniThFAST, minThFAST)
            const Arr &dims = get(in, "D.dims");
            const int levels = (int)dims.n / 2;
            ORBextractor ex;
            const uint8_t *sr = get(in, "D.raw").p<uint8_t>();
            for (int l = 0; l < levels; l++) {
                const int rows = dims.p<int32_t>()[2 * l], cols = dims.p<int32_t>()[2 * l + 1];
                cv::Mat m(rows, cols, (size_t)cols + 5);
                for (int r = 0; r < rows; r++) std::memcpy(m.ptr<unsigned char>(r), sr + (size_t)r * cols, cols);
                sr += (size_t)rows * cols;
                ex.mvImagePyramid.push_back(std::move(m));
            }
            const Arr &nf = get(in, "D.nf"), &sc = get(in, "D.scale"), &th = get(in, "D.th");
            std::vector<int> nfl(nf.p<int32_t>(), nf.p<int32_t>() + nf.n);
            std::vector<float> scl(sc.p<float>(), sc.p<float>() + sc.n);
            std::vector<std::vector<cv::KeyPoint>> all;
            const int n = osg_orbslam3::compute_keypoints_oct_tree(ex.mvImagePyramid, all, nfl, scl, th.p<int32_t>()[0],
                                                                  th.p<int32_t>()[1]);
            std::vector<float> x, y, r, sz, a;
            std::vector<int32_t> oct;
            for (auto &lv : all)
                for (auto &kp : lv) {
                    x.push_back(kp.pt.x);
                    y.push_back(kp.pt.y);
                    r.push_back(kp.response);
                    sz.push_back(kp.size);
                    a.push_back(kp.angle);
                    oct.push_back(kp.octave);
                }
            out["n"] = make('i', std::vector<int32_t>{n});
            out["x"] = make('f', x);
            out["y"] = make('f', y);
            out["response"] = make('f', r);
            out["size"] = make('f', sz);
            out["angle"] = make('f', a);
            out["octave"] = make('i', oct);
        } else if (mode == "distinct") {
            // keyframes: "K.desc" (nk x nkp rows), "K.bad"; MapPoints: "M.bad", "M.desc" (initial);
            // observations CSR "O.start" / "O.kf" / "O.left" / "O.right"
            const int nk = (int)get(in, "K.bad").n, nm = (int)get(in, "M.bad").n;
            const int nkp = (int)(get(in, "K.desc").n / 32 / (nk ? nk : 1));
            std::vector<KeyFrame> K(nk);
            for (int k = 0; k < nk; k++) {
                K[k].N = nkp;
                K[k].bad = get(in, "K.bad").p<uint8_t>()[k];
                K[k].mDescriptors = cv::Mat(nkp, 32);
                std::memcpy(K[k].mDescriptors.buf.data(), get(in, "K.desc").p<uint8_t>() + (size_t)k * nkp * 32,
                            (size_t)nkp * 32);
            }
            std::vector<MapPoint> M(nm);
            std::vector<MapPoint *> list;
            const int32_t *os = get(in, "O.start").p<int32_t>();
            for (int i = 0; i < nm; i++) {
                M[i].mnId = (unsigned long)i;
                M[i].bad = get(in, "M.bad").p<uint8_t>()[i];
                std::memcpy(M[i].desc.buf.data(), get(in, "M.desc").p<uint8_t>() + 32 * (size_t)i, 32);
                for (int o = os[i]; o < os[i + 1]; o++)
                    M[i].obs[&K[get(in, "O.kf").p<int32_t>()[o]]] =
                        std::make_tuple(get(in, "O.left").p<int32_t>()[o], get(in, "O.right").p<int32_t>()[o]);
                list.push_back(i % 17 == 5 ? nullptr : &M[i]);  // a NULL entry now and then
            }
            osg_orbslam3::compute_distinctive_descriptors<MockHooks>(list);
            std::vector<uint8_t> d(32 * (size_t)nm);
            for (int i = 0; i < nm; i++) std::memcpy(&d[32 * (size_t)i], M[i].desc.buf.data(), 32);
            out["desc"] = make('b', d);
        } else {
            fprintf(stderr, "unknown mode %s\n", mode.c_str());
            return 2;
        }
        write_arrays(argv[3], out);
    } catch (const std::exception &e) {
        fprintf(stderr, "adapter_driver: %s\n", e.what());
        return 1;
    }
    return 0;
}
