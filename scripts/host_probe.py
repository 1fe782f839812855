import os, time, json
import torch
info = {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us"):
    try:
        info[f] = open(f).read().strip()
    except OSError:
        pass
a = torch.randn(2048, 2048); b = torch.randn(2048, 2048)
for th in (8, 16, 32, 64, info["affinity"]):
    torch.set_num_threads(th)
    a @ b
    t = time.perf_counter()
    for _ in range(10):
        a @ b
    dt = (time.perf_counter() - t) / 10
    info[f"mm_tflops_{th}"] = 2 * 2048**3 / dt / 1e12
print(json.dumps(info))
