"""Per-configuration timing of the top-2 tile kernel; one child process per configuration because
the launch knobs (OSG_TOP2_*) are read once per process.  The parent never touches the GPU.

    python tools/top2_breakdown.py nq nt "VARIANT:WAVES:WG:DEBUG[:STREAM_G[:QT]]" ...

Each child prints one JSON line: per-launch event bracket, empty bracket, and back-to-back
average, so the event calibration can be compared with rocprofv3 --kernel-trace."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.environ["OSG_ROOT"])
from orb_slam3_comments_ghr_amd import Context, synth
nq, nt = int(sys.argv[1]), int(sys.argv[2])
dev = torch.device("cuda", 0)
stream = torch.cuda.Stream(dev); torch.cuda.set_stream(stream)
ctx = Context(0); ctx.set_stream(stream.cuda_stream)
if nt >= (1 << 20):  # C2'-sized: generate on the device (as bench.py does)
    g = torch.Generator(device=dev); g.manual_seed(synth.SEED_C2_STREAM)
    dt = torch.randint(0, 256, (nt, 32), dtype=torch.uint8, device=dev, generator=g)
    dq = torch.randint(0, 256, (nq, 32), dtype=torch.uint8, device=dev, generator=g)
else:
    q, t = synth.descriptors_c2(nq, nt)
    dq = torch.from_numpy(q).to(dev); dt = torch.from_numpy(t).to(dev)
dout = torch.empty((nq, 3), dtype=torch.int32, device=dev)
def run(): ctx.hamming_top2_dev(dq, nq, dt, nt, dout)
for _ in range(20): run()
torch.cuda.synchronize()
n = 300 if nt < (1 << 20) else 20
def brackets(body):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    torch.cuda._sleep(int(2e6 + n * 2e4))
    for a, b in evs:
        a.record(stream); body(); b.record(stream)
    torch.cuda.synchronize()
    return np.array([a.elapsed_time(b) for a, b in evs]) * 1e3
k = brackets(run)
e = brackets(lambda: None)
s = torch.cuda.Event(enable_timing=True); f = torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(int(2e6 + n * 2e4))
s.record(stream)
for _ in range(n): run()
f.record(stream); torch.cuda.synchronize()
ok = None
if os.environ.get("OSG_TOP2_DEBUG", "0") == "0":
    got = dout.cpu().numpy()
    ref = np.load(os.path.join(os.environ["OSG_ROOT"], "gpurun_out", "ref_%d_%d.npy" % (nq, nt))) if os.path.exists(os.path.join(os.environ["OSG_ROOT"], "gpurun_out", "ref_%d_%d.npy" % (nq, nt))) else None
    if ref is None:
        np.save(os.path.join(os.environ["OSG_ROOT"], "gpurun_out", "ref_%d_%d.npy" % (nq, nt)), got)
    else:
        ok = bool((ref == got).all())
print(json.dumps({"bracket_us": float(k.mean()), "bracket_med_us": float(np.median(k)), "empty_us": float(e.mean()),
                  "b2b_us": float(s.elapsed_time(f) * 1e3 / n), "same_as_first_cfg": ok}))
'''


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    nq, nt = sys.argv[1], sys.argv[2]
    for cfg in sys.argv[3:]:
        f = cfg.split(":")
        variant, waves, wg, dbg = f[:4]
        env = dict(os.environ, OSG_ROOT=root, OSG_TOP2_VARIANT=variant, OSG_TOP2_WAVES=waves,
                   OSG_TOP2_WG=wg, OSG_TOP2_QS_WG=wg, OSG_TOP2_DEBUG=dbg)
        if len(f) > 4 and f[4]:
            env["OSG_TOP2_STREAM_G"] = f[4]
        if len(f) > 5 and f[5]:
            env["OSG_TOP2_QT"] = f[5]
        r = subprocess.run([sys.executable, "-c", CHILD, nq, nt], env=env, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else json.dumps({"rc": r.returncode, "err": r.stderr[-400:]})
        print(json.dumps({"nq": int(nq), "nt": int(nt), "cfg": cfg, **json.loads(line)}), flush=True)


if __name__ == "__main__":
    main()
