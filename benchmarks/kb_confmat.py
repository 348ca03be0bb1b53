import os, sys, json, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from benchmarks.kbench import timeit, case_confmat
from torchmetrics_amd import ops
r = case_confmat()
N, C = 8192, 1000
x = [torch.randn(N, C, device="cuda").to(torch.bfloat16) for _ in range(4)]
it = [0]
def rd():
    i = it[0] = (it[0] + 1) % 4
    return x[i].amax(1)
def cl():
    i = it[0] = (it[0] + 1) % 4
    return x[i].clone()
r["amax_us"] = round(timeit(rd), 2)
r["clone_us"] = round(timeit(cl), 2)
r["lpr"] = os.environ.get("TM_AMD_MC_LPR", "auto")
print(json.dumps(r))
