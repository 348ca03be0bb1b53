"""Diagnostic: why does the native forward decline after a first Python forward?  Prints what
csrc/bindings/fastcall.cpp ``forward_allowed`` / ``states_unobserved`` / ``workspace`` look at."""
import gc
import sys

import torch

import torchmetrics_amd as tm


def report(m, keys):
    d = m.__dict__
    print("  flags:", {k: d.get(k) for k in ("_is_synced", "dist_sync_on_step", "compute_on_cpu", "validate_args",
                                              "multidim_average", "top_k", "average", "normalize")})
    print("  flag identities:", d.get("_is_synced") is False, d.get("dist_sync_on_step") is False,
          d.get("compute_on_cpu") is False)
    err = d.get("_device_errors")
    print("  err word:", None if err is None else (err.device, err.dtype))
    ws = d.get("_ws")
    print("  ws:", type(ws).__name__, None if ws is None else [(k, tuple(v.shape), v.dtype) for k, v in vars(ws).items()
                                                               if isinstance(v, torch.Tensor)] if hasattr(ws, "__dict__") else ws)
    for k in keys:
        t = d[k]
        stor = t.untyped_storage()
        uc = torch._C._storage_Use_Count(stor._cdata) - 1
        sharing = [a for a, v in d.items() if isinstance(v, torch.Tensor) and v.untyped_storage().data_ptr() == stor.data_ptr()]
        base = t._base
        print(f"  {k}: refcnt={sys.getrefcount(t) - 1} view={base is not None} use_count={uc} shape={tuple(t.shape)}"
              f" dtype={t.dtype} contig={t.is_contiguous()} sharing={sharing}")
        refs = [type(r).__name__ + (":" + ",".join(list(r.keys())[:6]) if isinstance(r, dict) else "")
                for r in gc.get_referrers(t)]
        print("     referrers:", refs)
        del stor


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    for name, make, keys in (("confmat", lambda: tm.MulticlassConfusionMatrix(5), ["confmat"]),
                             ("acc10", lambda: tm.classification.MulticlassAccuracy(10), ["tp", "fp", "tn", "fn"]),
                             ("binacc", lambda: tm.classification.BinaryAccuracy(), ["tp", "fp", "tn", "fn"])):
        m = make().to(dev)
        C = getattr(m, "num_classes", None)
        print(name, "forward type:", type(m.forward).__name__)
        for i in range(3):
            if C:
                p, t = torch.randn(513, C, generator=g), torch.randint(0, C, (513,), generator=g)
            else:
                p, t = torch.rand(513, generator=g), torch.randint(0, 2, (513,), generator=g)
            print(f" before call {i}:")
            report(m, keys)
            m(p.to(dev), t.to(dev))
            print(f" after call {i}: native_calls={m.forward.native_calls} decline_line={m.forward.decline_line}")


if __name__ == "__main__":
    main()
