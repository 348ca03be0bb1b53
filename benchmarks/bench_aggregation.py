"""Aggregator and exact-match updates: the one-launch ``agg_update`` kernel (``csrc/common/aggregate.hip``) vs the reference's op
chain (``S/aggregation.py:75-105`` + ``MeanMetric.update`` ``:550-575``: as_tensor weight, broadcast, isnan x2,
``nans.any()`` host check, cast, ``(x * w).sum()``, ``w.sum()``, in-place adds), same inputs, same process.
Exact match (``csrc/classification/exact_match.hip``) vs the reference's chain (``F/classification/exact_match.py``:
argmax / ``_prob_or`` host check + sigmoid + threshold, ``==``, ``.sum(1) == L``, ``.sum()``).
One JSON line per case: ours_us / reference_us per update (wall clock over a loop of updates, then one sync)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402


def ref_mean_update(state, value, weight=1.0):
    dtype = state[0].dtype
    if not isinstance(weight, torch.Tensor):
        weight = torch.as_tensor(weight, dtype=dtype, device=value.device)
    weight = torch.broadcast_to(weight, value.shape)
    nans, nans_w = torch.isnan(value), torch.isnan(weight)
    if nans.any() or nans_w.any():  # host sync, as in the reference
        keep = ~(nans | nans_w)
        value, weight = value[keep], weight[keep]
    value, weight = value.to(dtype), weight.to(dtype)
    if value.numel() == 0:
        return
    state[0] += (value * weight).sum()
    state[1] += weight.sum()


def loop_us(fn, xs, reps):
    for x in xs[:3]:
        fn(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(xs[i % len(xs)])
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / reps


def hbm_tb_s(nbytes, us):
    return round(nbytes / (us * 1e-6) / 1e12, 2)


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for n, label in ((1, "scalar loss"), (4096, "4096 per-sample losses"), (16_777_216, "16.8M values")):
        xs = [torch.randn(n, device=dev, generator=g) for _ in range(8)]
        reps = 200 if n < 1_000_000 else 50
        ours = tm.MeanMetric().to(dev)
        t_ours = loop_us(ours.update, xs, reps)
        state = [torch.zeros((), device=dev), torch.zeros((), device=dev)]
        t_ref = loop_us(lambda x: ref_mean_update(state, x), xs, reps)
        chk_o = tm.MeanMetric().to(dev)
        chk_r = [torch.zeros((), device=dev, dtype=torch.float64), torch.zeros((), device=dev, dtype=torch.float64)]
        for x in xs:
            chk_o.update(x)
            ref_mean_update(chk_r, x.double())
        diff = abs(float(chk_o.compute()) - float(chk_r[0] / chk_r[1]))
        print(json.dumps({"case": f"MeanMetric.update {label}", "ours_us": round(t_ours, 2),
                          "reference_us": round(t_ref, 2), "speedup": round(t_ref / t_ours, 2),
                          "ours_effective_TB_s": hbm_tb_s(4 * n, t_ours), "abs_diff_vs_fp64": diff}), flush=True)
    xs = [torch.randn(4096, device=dev, generator=g) for _ in range(8)]
    for name, cls in (("SumMetric", tm.SumMetric), ("MaxMetric", tm.MaxMetric)):
        m = cls(nan_strategy="ignore").to(dev)
        t = loop_us(m.update, xs, 200)
        print(json.dumps({"case": f"{name}(nan_strategy='ignore').update 4096", "ours_us": round(t, 2)}), flush=True)
    exact_match_cases(dev, g)


def ref_multiclass_em(state, preds, target):
    p = preds.argmax(1).reshape(preds.shape[0], -1)
    t = target.reshape(target.shape[0], -1)
    state[0] += ((p == t).sum(1) == p.shape[1]).sum()
    state[1] += p.shape[0]


def ref_multilabel_em(state, preds, target, threshold=0.5):
    if not torch.all((preds >= 0) * (preds <= 1)):  # host sync, as the reference's _prob_or check
        preds = preds.sigmoid()
    p = (preds > threshold).long()
    state[0] += ((p == target).sum(1) == p.shape[1]).sum()
    state[1] += p.shape[0]


def exact_match_cases(dev, g):
    for label, c, dtype in (("65536x1000 bf16", 1000, torch.bfloat16), ("65536x10 f32", 10, torch.float32)):
        xs = [(torch.randn(65536, c, device=dev, generator=g).to(dtype),
               torch.randint(0, c, (65536,), device=dev, generator=g)) for _ in range(4)]
        m = tm.MulticlassExactMatch(c).to(dev)
        t_ours = loop_us(lambda a: m.update(*a), xs, 100)
        st = [torch.zeros((), dtype=torch.long, device=dev), torch.zeros((), dtype=torch.long, device=dev)]
        t_ref = loop_us(lambda a: ref_multiclass_em(st, *a), xs, 100)
        print(json.dumps({"case": f"MulticlassExactMatch.update {label}", "ours_us": round(t_ours, 2),
                          "reference_us": round(t_ref, 2), "speedup": round(t_ref / t_ours, 2),
                          "ours_effective_TB_s": hbm_tb_s(xs[0][0].numel() * xs[0][0].element_size(), t_ours)}),
              flush=True)
    xs = [(torch.randn(65536, 64, device=dev, generator=g), torch.randint(0, 2, (65536, 64), device=dev, generator=g))
          for _ in range(4)]
    m = tm.MultilabelExactMatch(64).to(dev)
    t_ours = loop_us(lambda a: m.update(*a), xs, 100)
    st = [torch.zeros((), dtype=torch.long, device=dev), torch.zeros((), dtype=torch.long, device=dev)]
    t_ref = loop_us(lambda a: ref_multilabel_em(st, *a), xs, 100)
    print(json.dumps({"case": "MultilabelExactMatch.update 65536x64 logits", "ours_us": round(t_ours, 2),
                      "reference_us": round(t_ref, 2), "speedup": round(t_ref / t_ours, 2),
                      "ours_effective_TB_s": hbm_tb_s(65536 * 64 * 12, t_ours)}), flush=True)


if __name__ == "__main__":
    main()
