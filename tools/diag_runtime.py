import sys, os, subprocess
code1 = r'''
import sys; sys.path.insert(0, "mpc-tsid_amd")
MODE = sys.argv[1]
if MODE == "torch_first":
    import torch
import mpcq
e = mpcq.Engine(16)
import torch
try:
    t = torch.zeros(4, device="cuda"); print(MODE, "torch ok", t.device)
except Exception as ex:
    print(MODE, "torch FAIL", ex)
libs = sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l})
print(MODE, libs)
'''
for m in ("mpcq_first", "torch_first"):
    r = subprocess.run([sys.executable, "-c", code1, m], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr[-500:])
