import os
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for p in ["/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective"]:
    try: print(p, open(p).read().strip())
    except Exception as e: print(p, e)
print(open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0])
