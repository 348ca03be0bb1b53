"""Op-for-op emulation of the reference's ``MulticlassConfusionMatrix`` hot path, used as the in-run baseline.

The reference (torchmetrics 1.4.0dev) cannot be imported on the GPU box (its ``lightning_utilities`` dependency is not
installed and the repo is not shipped there), so ``bench.py`` re-creates its exact torch-op sequence:

update (``S/classification/confusion_matrix.py:284-289`` -> ``F/classification/confusion_matrix.py``):
  1. ``_multiclass_confusion_matrix_tensor_validation``: ``len(torch.unique(target))`` (device->host sync)
     (``F/classification/confusion_matrix.py`` -> ``stat_scores.py:307``); float preds skip the preds check.
  2. ``_multiclass_confusion_matrix_format``: ``preds.argmax(dim=1)``, flatten, ignore_index mask (none here).
  3. ``_multiclass_confusion_matrix_update``: ``torch.bincount(target*C + preds, minlength=C*C).reshape(C, C)``.
  4. ``self.confmat += confmat``.

sync (``S/metric.py:427-457`` + ``S/utilities/distributed.py:97-147``), per state tensor:
  ``barrier`` -> ``all_gather(shape)`` -> ``all_gather(data)`` -> ``torch.stack`` -> ``sum(dim=0)``.
"""
from typing import List

import torch
import torch.distributed as dist
from torch import Tensor


class ReferenceEmulatedConfusionMatrix:
    def __init__(self, num_classes: int, device: torch.device) -> None:
        self.num_classes = num_classes
        self.confmat = torch.zeros(num_classes, num_classes, dtype=torch.long, device=device)

    def update(self, preds: Tensor, target: Tensor) -> None:
        c = self.num_classes
        # validation: unique-count check (host sync) as in the reference tensor validation
        n_unique = len(torch.unique(target))
        if n_unique > c:
            raise RuntimeError("Detected more unique values in `target` than `num_classes`.")
        # format
        labels = preds.argmax(dim=1).flatten()
        tgt = target.flatten()
        # update
        mapping = tgt.to(torch.long) * c + labels.to(torch.long)
        bins = torch.bincount(mapping, minlength=c * c)
        self.confmat += bins.reshape(c, c)

    def _gather_all_tensors(self, result: Tensor) -> List[Tensor]:
        result = result.contiguous()
        world = dist.get_world_size()
        dist.barrier()
        local_size = torch.tensor(result.shape, device=result.device)
        sizes = [torch.zeros_like(local_size) for _ in range(world)]
        dist.all_gather(sizes, local_size)
        out = [torch.zeros_like(result) for _ in range(world)]
        dist.all_gather(out, result)
        return out

    def compute(self) -> Tensor:
        if dist.is_available() and dist.is_initialized():
            gathered = self._gather_all_tensors(self.confmat)
            return torch.stack(gathered).sum(dim=0)
        return self.confmat


# --------------------------------------------------------------------------------------------------- config #5
def _ref_gather_reduce(t: Tensor, op: str = "sum") -> Tensor:
    """One state through the reference sync: barrier + all_gather(shape) + all_gather(data) + stack + reduce
    (``S/utilities/distributed.py:97-147`` then ``dim_zero_*``, ``S/metric.py:442-457``)."""
    if not (dist.is_available() and dist.is_initialized()):
        return t
    w = dist.get_world_size()
    t = t.contiguous()
    dist.barrier()
    shape = torch.tensor(t.shape, device=t.device)
    shapes = [torch.zeros_like(shape) for _ in range(w)]
    dist.all_gather(shapes, shape)
    out = [torch.zeros_like(t) for _ in range(w)]
    dist.all_gather(out, t)
    st = torch.stack(out)
    return st.sum(0) if op == "sum" else torch.cat(out)


def _safe_divide(num: Tensor, den: Tensor) -> Tensor:
    den = den.clone()
    den[den == 0.0] = 1  # reference _safe_divide (S/utilities/compute.py:46-55), in-place on the denominator
    return num.float() / den.float()


class ReferenceEmulatedCollection:
    """Op-for-op emulation of the reference ``MetricCollection`` of bench_collection.py's 20 metrics with
    ``compute_groups=True`` (``S/collections.py:200-359``): ONE update per compute group (stat scores, confusion
    matrix, binned multiclass PR curve, calibration lists, and the five regression metrics), and a ``compute()`` in
    which EVERY metric syncs each of its own states separately before its reduce.

    Update chains (reference functional code):
      * stat scores / confmat: tensor validation ``len(torch.unique(target))`` (host sync), ``argmax``,
        ``bincount(target * C + preds)`` (``F/classification/stat_scores.py:281-448``,
        ``F/classification/confusion_matrix.py:333-337``);
      * binned PR curve, 100 thresholds: ``torch.all(0 <= preds <= 1)`` (host sync) -> softmax, the vectorised
        ``[N, C, T]`` threshold compare + ``bincount`` (``F/classification/precision_recall_curve.py:482-527``);
      * calibration: prob check (host sync), softmax, ``max(1)``, ``eq`` appended to lists
        (``F/classification/calibration_error.py``);
      * MSE / MAE / R2 / Pearson / explained variance: their moment updates (``F/regression/*.py``).
    """

    def __init__(self, num_classes: int, device: torch.device, thresholds: int = 100, n_bins: int = 15) -> None:
        self.c, self.dev, self.n_bins = num_classes, device, n_bins
        self.thr = torch.linspace(0, 1, thresholds, device=device)
        self.reset()

    def reset(self) -> None:
        c, dev, t = self.c, self.dev, self.thr.numel()
        z = lambda *s, dt=torch.long: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        self.tp, self.fp, self.tn, self.fn = z(c), z(c), z(c), z(c)
        self.confmat = z(c, c)
        self.curve = z(t, c, 2, 2)
        self.conf, self.accs = [], []
        f = lambda: torch.zeros((), device=dev)  # noqa: E731
        self.mse_sse, self.mse_n = f(), z(())
        self.mae_sae, self.mae_n = f(), z(())
        self.r2 = [f(), f(), f(), z(())]
        self.pearson = [f() for _ in range(5)] + [f()]
        self.ev = [z(()), f(), f(), f(), f()]

    def _check_target(self, target: Tensor) -> None:
        if len(torch.unique(target)) > self.c:
            raise RuntimeError("more unique values in target than num_classes")

    def update_cls(self, preds: Tensor, target: Tensor) -> None:
        c = self.c
        # stat-score group (accuracy ... stat scores)
        self._check_target(target)
        lab = preds.argmax(1)
        cm = torch.bincount(target.long() * c + lab.long(), minlength=c * c).reshape(c, c)
        tp = cm.diag()
        fp = cm.sum(0) - tp
        fn = cm.sum(1) - tp
        tn = cm.sum() - (fp + fn + tp)
        self.tp += tp
        self.fp += fp
        self.tn += tn
        self.fn += fn
        # confusion-matrix group (jaccard, mcc, kappa, confmat)
        self._check_target(target)
        lab = preds.argmax(1)
        self.confmat += torch.bincount(target.long() * c + lab.long(), minlength=c * c).reshape(c, c)
        # binned PR-curve group (auroc, average precision)
        self._check_target(target)
        p = preds
        if not torch.all((p >= 0) * (p <= 1)):
            p = p.softmax(1)
        t = self.thr.numel()
        preds_t = (p.unsqueeze(-1) >= self.thr.unsqueeze(0).unsqueeze(0)).long()
        target_t = torch.nn.functional.one_hot(target, num_classes=c)
        mapping = preds_t + 2 * target_t.unsqueeze(-1) + 4 * torch.arange(c, device=p.device).unsqueeze(0).unsqueeze(-1) \
            + 4 * c * torch.arange(t, device=p.device)
        self.curve += torch.bincount(mapping.flatten(), minlength=4 * c * t).reshape(t, c, 2, 2)
        # calibration error
        self._check_target(target)
        p = preds
        if not torch.all((p >= 0) * (p <= 1)):
            p = p.softmax(1)
        conf, pred = p.max(dim=1)
        self.conf.append(conf.float())
        self.accs.append(pred.eq(target).float())

    def update_reg(self, preds: Tensor, target: Tensor) -> None:
        diff = preds - target
        self.mse_sse += torch.sum(diff * diff)
        self.mse_n += target.numel()
        self.mae_sae += torch.sum(torch.abs(diff))
        self.mae_n += target.numel()
        r = target - preds
        self.r2[0] += torch.sum(r * r)
        self.r2[1] += target.sum(0)
        self.r2[2] += (target * target).sum(0)
        self.r2[3] += target.numel()
        # pearson (F/regression/pearson.py:25-78): running means / variances / covariance
        mx, my, vx, vy, cxy, n = self.pearson
        n_obs = preds.shape[0]
        mx_new = (n * mx + preds.sum(0)) / (n + n_obs)
        my_new = (n * my + target.sum(0)) / (n + n_obs)
        n_new = n + n_obs
        vx += ((preds - mx_new) * (preds - mx)).sum(0)
        vy += ((target - my_new) * (target - my)).sum(0)
        cxy += ((preds - mx) * (target - my_new)).sum(0)
        self.pearson = [mx_new, my_new, vx, vy, cxy, n_new]
        e = self.ev
        e[0] += target.shape[0]
        e[1] += r.sum(0)
        e[2] += (r * r).sum(0)
        e[3] += target.sum(0)
        e[4] += (target * target).sum(0)

    def compute(self) -> dict:
        g = _ref_gather_reduce
        out = {}
        # 8 stat-score metrics, each syncing its own 4 states
        for name in ("acc", "prec", "rec", "f1", "fbeta", "spec", "hamming", "stat"):
            tp, fp, tn, fn = g(self.tp), g(self.fp), g(self.tn), g(self.fn)
            if name == "acc" or name == "rec":
                score = _safe_divide(tp, tp + fn)
            elif name == "prec":
                score = _safe_divide(tp, tp + fp)
            elif name in ("f1", "fbeta"):
                b2 = 1.0 if name == "f1" else 4.0
                score = _safe_divide((1 + b2) * tp, (1 + b2) * tp + b2 * fn + fp)
            elif name == "spec":
                score = _safe_divide(tn, tn + fp)
            elif name == "hamming":
                score = 1 - _safe_divide(tp, tp + fn)
            else:
                out[name] = torch.stack([tp, fp, tn, fn, tp + fn], dim=-1).sum(0)
                continue
            w = torch.ones_like(score)
            w[tp + fp + fn == 0] = 0.0
            out[name] = _safe_divide(w * score, w.sum(-1, keepdim=True)).sum(-1)
        # 4 confusion-matrix metrics
        for name in ("jacc", "mcc", "kappa", "cm"):
            cm = g(self.confmat).float()
            if name == "jacc":
                inter = cm.diag()
                union = cm.sum(0) + cm.sum(1) - inter
                out[name] = _safe_divide(inter, union).mean()
            elif name == "mcc":
                tk, pk = cm.sum(1), cm.sum(0)
                cc, s = cm.trace(), cm.sum()
                out[name] = (cc * s - (tk * pk).sum()) / (torch.sqrt(s**2 - (pk * pk).sum()) * torch.sqrt(s**2 - (tk * tk).sum()))
            elif name == "kappa":
                n = cm.sum()
                po = cm.trace() / n
                pe = (cm.sum(0) * cm.sum(1)).sum() / n**2
                out[name] = 1 - (1 - po) / (1 - pe)
            else:
                out[name] = cm
        # binned AUROC / AP from the [T, C, 2, 2] state
        for name in ("auroc", "ap"):
            st = g(self.curve)
            tps, fps, fns = st[:, :, 1, 1], st[:, :, 0, 1], st[:, :, 1, 0]
            tns = st[:, :, 0, 0]
            prec = _safe_divide(tps, tps + fps)
            rec = _safe_divide(tps, tps + fns)
            if name == "auroc":
                fpr = _safe_divide(fps, fps + tns).flip(0)
                tpr = rec.flip(0)
                out[name] = torch.trapz(tpr, fpr, dim=0).mean()
            else:
                prec = torch.cat([prec, torch.ones(1, prec.shape[1], device=prec.device)])
                rec = torch.cat([rec, torch.zeros(1, rec.shape[1], device=rec.device)])
                out[name] = (-(rec[1:] - rec[:-1]) * prec[:-1]).sum(0).mean()
        conf = g(torch.cat(self.conf), "cat")
        accs = g(torch.cat(self.accs), "cat")
        bounds = torch.linspace(0, 1, self.n_bins + 1, device=conf.device)
        idx = torch.bucketize(conf, bounds, right=True) - 1
        cnt = torch.zeros(self.n_bins, device=conf.device).scatter_add_(0, idx.clamp(max=self.n_bins - 1), torch.ones_like(conf))
        sc = torch.zeros(self.n_bins, device=conf.device).scatter_add_(0, idx.clamp(max=self.n_bins - 1), conf)
        sa = torch.zeros(self.n_bins, device=conf.device).scatter_add_(0, idx.clamp(max=self.n_bins - 1), accs)
        out["ece"] = (torch.nan_to_num(sa / cnt) - torch.nan_to_num(sc / cnt)).abs().mul(cnt / cnt.sum()).sum()
        sse, n = g(self.mse_sse), g(self.mse_n)
        out["mse"] = sse / n
        sae, n = g(self.mae_sae), g(self.mae_n)
        out["mae"] = sae / n
        rss, s, ss, n = (g(x) for x in self.r2)
        out["r2"] = 1 - rss / (ss - s * s / n)
        mx, my, vx, vy, cxy, n = (g(x) for x in self.pearson)
        out["pearson"] = cxy / (vx * vy).sqrt()
        n, se, sse, st, sst = (g(x) for x in self.ev)
        out["ev"] = 1 - ((sse - se * se / n) / n) / ((sst - st * st / n) / n)
        return out
