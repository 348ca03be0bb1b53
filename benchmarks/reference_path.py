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
