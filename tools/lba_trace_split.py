"""Per-kernel device time of a rocprofv3 kernel trace, split by batch size (Grid_Size_Y = graphs).
usage: python tools/lba_trace_split.py <kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(lambda: [0, 0.0])
steps = collections.Counter()
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    gy = int(r["Grid_Size_Y"])
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by[(gy, name)][0] += 1
    by[(gy, name)][1] += dur
    if name == "k_step_reduce":
        steps[gy] += 1
for gy in sorted({k[0] for k in by}):
    items = sorted(((v[1], k[1], v[0]) for k, v in by.items() if k[0] == gy), reverse=True)
    tot = sum(i[0] for i in items)
    n = max(steps[gy], 1)
    print(f"grid.y={gy}: {n} steps, device {tot / n:.1f} us per step")
    for t, name, c in items[:14]:
        print(f"   {name:28s} {c:6d} launches  {t / n:9.1f} us/step  {100 * t / tot:5.1f} %")
