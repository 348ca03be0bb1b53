"""``metric(preds, target)`` (forward: batch value + accumulation) on ROCm, 8192 x 1000 bf16 logits.

Three implementations of the same forward, in one process, on the same data:

* ``native``: the C++ ``NativeForward`` (``csrc/bindings/fastcall.cpp``; stat scores fold + score in one launch,
  ``csrc/classification/forward.hip``);
* ``python``: ``Metric.forward`` of this package (batch reset / update / compute / merge in Python);
* ``reference``: an op-for-op emulation of the reference's ``_forward_reduce_state_update``
  (``S/metric.py:275-306,353-391``): save the global states, reset (clone every default), update (tensor validation
  with its ``torch.unique`` host sync, argmax, bincount, diag / sum algebra), compute (``_safe_divide`` /
  ``_adjust_weights_safe_divide``), then ``global + batch`` per state.

Every batch value and the final accumulated state are checked equal across the three.  One JSON line per metric;
``vs_baseline`` = reference time / native time.  Usage: ``python benchmarks/bench_forward.py [--steps K]``.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402

N, C = 8192, 1000


class _RefForward:
    """The reference's reduce-state forward for MulticlassConfusionMatrix / MulticlassAccuracy(average='macro')."""

    def __init__(self, kind: str, device: torch.device) -> None:
        self.kind = kind
        z = lambda *s: torch.zeros(*s, dtype=torch.long, device=device)  # noqa: E731
        self.defaults = {"confmat": z(C, C)} if kind == "confmat" else {k: z(C) for k in ("tp", "fp", "tn", "fn")}
        self.state = {k: v.clone() for k, v in self.defaults.items()}

    def _update(self, st, preds, target):
        if len(torch.unique(target)) > C:  # _multiclass_*_tensor_validation (host sync)
            raise RuntimeError("Detected more unique values in `target` than `num_classes`.")
        lab = preds.argmax(dim=1)
        cm = torch.bincount(target.long() * C + lab.long(), minlength=C * C).reshape(C, C)
        if self.kind == "confmat":
            st["confmat"] += cm
            return
        tp = cm.diag()
        fp = cm.sum(0) - tp
        fn = cm.sum(1) - tp
        tn = cm.sum() - (fp + fn + tp)
        st["tp"] += tp
        st["fp"] += fp
        st["tn"] += tn
        st["fn"] += fn

    def _compute(self, st):
        if self.kind == "confmat":
            return st["confmat"]
        tp, fn, fp = st["tp"], st["fn"], st["fp"]
        den = (tp + fn).clone()
        den[den == 0] = 1
        score = tp.float() / den.float()
        w = torch.ones_like(score)
        w[tp + fp + fn == 0] = 0.0
        wsum = w.sum(-1, keepdim=True)
        wsum[wsum == 0] = 1
        return (w * score / wsum).sum(-1)

    def __call__(self, preds, target):
        glob = self.state
        batch = {k: v.detach().clone() for k, v in self.defaults.items()}  # reset()
        self._update(batch, preds, target)
        val = self._compute(batch)
        self.state = {k: glob[k] + batch[k] for k in glob}  # _reduce_states: global + local
        return val


def _time(fn, preds, target, steps, keep=True):
    """Mean us per call; ``keep`` holds every returned value for the parity checks (for the confusion matrix that is
    an 8 MB tensor per call: the allocator grows by steps x 8 MB inside the timed loop)."""
    vals = []
    for i in range(10):
        fn(preds[i % len(preds)], target[i % len(target)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        v = fn(preds[i % len(preds)], target[i % len(target)])
        if keep:
            vals.append(v)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6, vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--ours-only", action="store_true",
                    help="only the native forward (attributable kernel traces: no Python / reference forwards)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    preds = [torch.randn(N, C, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4)]
    target = [torch.randint(0, C, (N,), device="cuda", generator=g) for _ in range(4)]
    cases = {
        "MulticlassConfusionMatrix(1000)": ("confmat", lambda: tm.MulticlassConfusionMatrix(C)),
        "MulticlassAccuracy(1000, macro)": ("acc", lambda: tm.MulticlassAccuracy(C)),
    }
    for name, (kind, make) in cases.items():
        native = make().to(dev)
        assert type(native.forward).__name__ == "NativeForward", type(native.forward)
        if args.ours_only:
            t_nat, _ = _time(native, preds, target, args.steps, keep=False)
            print(json.dumps({"metric": name, "batch": N, "dtype": "bf16", "steps": args.steps,
                              "forward_us": round(t_nat, 2), "native_calls": native.forward.native_calls}), flush=True)
            continue
        python = make().to(dev)
        python.__dict__.pop("forward")  # Metric.forward
        ref = _RefForward(kind, dev)
        t_nat, v_nat = _time(native, preds, target, args.steps)
        t_py, v_py = _time(python, preds, target, args.steps)
        t_ref, v_ref = _time(ref, preds, target, args.steps)
        for a, b, c in zip(v_nat, v_py, v_ref):
            if not (torch.equal(a, b) and torch.allclose(a.float(), c.float(), rtol=0, atol=1e-6)):
                raise RuntimeError(f"forward parity failure on {name}")
        final = native.compute()
        if not torch.allclose(final.float(), python.compute().float(), atol=1e-6):
            raise RuntimeError(f"accumulated state parity failure on {name}")
        print(json.dumps({
            "metric": name, "batch": N, "dtype": "bf16", "steps": args.steps,
            "forward_us": round(t_nat, 2), "python_forward_us": round(t_py, 2), "reference_forward_us": round(t_ref, 2),
            "vs_baseline": round(t_ref / t_nat, 2), "vs_python_forward": round(t_py / t_nat, 2),
            "native_calls": native.forward.native_calls,
            "baseline": "op-for-op emulation of the reference _forward_reduce_state_update (S/metric.py:353-391)",
        }), flush=True)


if __name__ == "__main__":
    main()
