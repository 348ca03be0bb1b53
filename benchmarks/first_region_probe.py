"""Fresh-process first-region cost of the headline loop (bench.py's exact shape: 406 MB ring, W warm-up updates,
compute, reset, sync, then ONE timed region of 20 updates + compute + sync).  Each case runs in its own process:

  python benchmarks/first_region_probe.py <case>   (case: plain | onering | onering_same5 | warm50 | sleep10ms ...)
Environment variables (e.g. HSA_ENABLE_INTERRUPT) are inherited from the caller.  Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd.classification import MulticlassConfusionMatrix  # noqa: E402

C, B, K = 1000, 8192, 26


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "plain"
    if case.startswith("sched_"):
        import ctypes

        flag = {"sched_spin": 1, "sched_yield": 2, "sched_blocking": 4}[case]
        rc = ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(flag)  # before the HIP context exists
        assert rc == 0, rc
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1234)
    if case.startswith("onering"):
        ring = torch.empty(K, B, C, dtype=torch.bfloat16, device=dev)
        for i in range(K):
            ring[i].copy_(torch.randn(B, C, generator=g, device=dev))
        preds = list(ring.unbind(0))
        target = list(torch.randint(0, C, (K, B), generator=g, device=dev).unbind(0))
    else:
        preds = [torch.randn(B, C, generator=g, device=dev).to(torch.bfloat16) for _ in range(K)]
        target = [torch.randint(0, C, (B,), generator=g, device=dev) for _ in range(K)]
    m = MulticlassConfusionMatrix(num_classes=C).to(dev)
    import gc

    if case == "nogc":
        gc.collect()
        gc.disable()
    warm = 50 if case == "warm50" else 5
    for i in range(warm):
        m.update(preds[i % K], target[i % K])
    if not case.endswith(("_nocr", "_ronly")):
        m.compute()
    if case.endswith("_zero"):  # the state zeroed by hand instead of reset()
        m.confmat.zero_()
        m._update_count = 0
        m._computed = None
    elif not case.endswith(("_nocr", "_conly")):
        tr = time.perf_counter()
        m.reset()  # (refills the state in place when unobserved)
        reset_us = (time.perf_counter() - tr) * 1e6
    torch.cuda.synchronize()
    if case == "sleep10ms":
        time.sleep(0.01)
    if case == "launches200":
        x = torch.zeros(1, device=dev)
        for _ in range(200):
            x.add_(1)
        torch.cuda.synchronize()
    if case == "cpuspin20":
        t_s = time.perf_counter()
        while time.perf_counter() - t_s < 0.02:
            pass
    if case in ("heavyspin20", "onering_heavy"):
        a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        t_s = time.perf_counter()
        while time.perf_counter() - t_s < 0.02:
            a = (a @ a).clamp_(-1, 1)
            torch.cuda.synchronize()
    if case in ("readring", "onering_read"):
        acc = torch.zeros((), device=dev)
        for p in preds:
            acc += p.float().sum()
        torch.cuda.synchronize()
    if case == "gpuspin20":
        x = torch.zeros(1, device=dev)
        t_s = time.perf_counter()
        while time.perf_counter() - t_s < 0.02:
            x.add_(1)
        torch.cuda.synchronize()
    out = {"case": case, "env_interrupt": os.environ.get("HSA_ENABLE_INTERRUPT"),
           "reset_us": round(reset_us, 1) if "reset_us" in locals() else None}
    for rep in range(3):
        torch.cuda.synchronize()
        gc0 = gc.get_count()
        ts = []
        t0 = time.perf_counter()
        for i in range(20):
            j = i % 5 if case.endswith("same5") else (5 + 20 * rep + i) % K  # same5: only the warm-up's 5 slots
            m.update(preds[j], target[j])
            ts.append(time.perf_counter())
        t1 = time.perf_counter()
        out[f"per_update{rep}"] = [round(1e6 * (b - a), 1) for a, b in zip([t0] + ts[:-1], ts)]
        out[f"gc{rep}"] = [gc0, gc.get_count()]
        m.compute()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        out[f"rep{rep}"] = [round(1e6 * (t3 - t0), 1), round(1e6 * (t1 - t0), 1), round(1e6 * (t2 - t1), 1),
                            round(1e6 * (t3 - t2), 1)]
        m.reset()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
