"""Multimodal metrics (reference ``F/multimodal/{clip_score,clip_iqa}.py``).

The CLIP encoders run through HuggingFace ``transformers`` on PyTorch-ROCm (their GEMMs are vendor MFMA GEMMs); the
metric math -- cosine of each (image, caption) embedding pair, the prompt-pair softmax of CLIP-IQA -- runs in one
wave-per-row kernel each on ROCm (``csrc/multimodal/clip.hip``).  Weights are never downloaded:
``model_name_or_path`` must resolve offline (a local directory or the HF cache).  The original CLIP-IQA network (``"clip_iqa"``) comes from ``piq`` and is gated on it.
"""
from typing import Dict, List, Literal, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.imports import _TRANSFORMERS_AVAILABLE
from torchmetrics_amd.utilities.prints import rank_zero_warn

_PROMPTS: Dict[str, Tuple[str, str]] = {
    "quality": ("Good photo.", "Bad photo."),
    "brightness": ("Bright photo.", "Dark photo."),
    "noisiness": ("Clean photo.", "Noisy photo."),
    "colorfullness": ("Colorful photo.", "Dull photo."),
    "sharpness": ("Sharp photo.", "Blurry photo."),
    "contrast": ("High contrast photo.", "Low contrast photo."),
    "complexity": ("Complex photo.", "Simple photo."),
    "natural": ("Natural photo.", "Synthetic photo."),
    "happy": ("Happy photo.", "Sad photo."),
    "scary": ("Scary photo.", "Peaceful photo."),
    "new": ("New photo.", "Old photo."),
    "warm": ("Warm photo.", "Cold photo."),
    "real": ("Real photo.", "Abstract photo."),
    "beautiful": ("Beautiful photo.", "Ugly photo."),
    "lonely": ("Lonely photo.", "Sociable photo."),
    "relaxing": ("Relaxing photo.", "Stressful photo."),
}


def _get_clip_model_and_processor(model_name_or_path: str = "openai/clip-vit-large-patch14"):
    if not _TRANSFORMERS_AVAILABLE:
        raise ModuleNotFoundError("`clip_score` metric requires `transformers` package be installed.")
    from transformers import CLIPModel, CLIPProcessor

    return CLIPModel.from_pretrained(model_name_or_path), CLIPProcessor.from_pretrained(model_name_or_path)


def _features(out) -> Tensor:
    """transformers < 5 returns the projected embedding tensor, >= 5 a ModelOutput whose ``pooler_output`` is it."""
    return out if isinstance(out, Tensor) else out.pooler_output


def _normalize(x) -> Tensor:
    x = _features(x)
    return x / x.norm(p=2, dim=-1, keepdim=True)


def _clip_score_update(images: Union[Tensor, List[Tensor]], text: Union[str, List[str]], model,
                       processor) -> Tuple[Tensor, int]:
    """Per-pair ``100 * cos(image embedding, caption embedding)`` and the number of pairs."""
    if not isinstance(images, list):
        images = [images] if images.ndim == 3 else list(images)
    if not all(i.ndim == 3 for i in images):
        raise ValueError("Expected all images to be 3d but found image that has either more or less")
    if not isinstance(text, list):
        text = [text]
    if len(text) != len(images):
        raise ValueError(
            f"Expected the number of images and text examples to be the same but got {len(images)} and {len(text)}")
    device = images[0].device
    proc = processor(text=text, images=[i.cpu() for i in images], return_tensors="pt", padding=True)
    img = _features(model.get_image_features(proc["pixel_values"].to(device)))
    max_pos = model.config.text_config.max_position_embeddings
    ids, am = proc["input_ids"], proc["attention_mask"]
    if am.shape[-1] > max_pos:
        rank_zero_warn(
            f"Encountered caption longer than max_position_embeddings={max_pos}. Will truncate captions to this length."
            "If longer captions are needed, initialize argument `model_name_or_path` with a model that supports"
            "longer sequences")
        ids, am = ids[..., :max_pos], am[..., :max_pos]
    txt = _features(model.get_text_features(ids.to(device), am.to(device)))
    return _scaled_cosine(img, txt, 100.0), len(text)


def _scaled_cosine(img: Tensor, txt: Tensor, scale: float) -> Tensor:
    """``scale * cos`` per embedding pair: one wave per pair on ROCm (``ops.paired_cosine``); the normalise-then-dot
    formulation of the reference when gradients are needed."""
    if img.is_cuda and not (torch.is_grad_enabled() and (img.requires_grad or txt.requires_grad)):
        return ops.paired_cosine(img, txt, scale).to(img.dtype)
    return scale * (_normalize(img) * _normalize(txt)).sum(dim=-1)


def clip_score(images: Union[Tensor, List[Tensor]], text: Union[str, List[str]],
               model_name_or_path: str = "openai/clip-vit-large-patch14") -> Tensor:
    """CLIPScore = max(100 cos(E_image, E_caption), 0), averaged over pairs (``F/multimodal/clip_score.py:104``)."""
    model, processor = _get_clip_model_and_processor(model_name_or_path)
    device = images.device if isinstance(images, Tensor) else images[0].device
    score, _ = _clip_score_update(images, text, model.to(device), processor)
    score = score.mean(0)
    return torch.max(score, torch.zeros_like(score))


def _get_clip_iqa_model_and_processor(model_name_or_path: str):
    if model_name_or_path == "clip_iqa":
        try:
            import piq
        except ImportError as err:
            raise ModuleNotFoundError(
                "For metric `clip_iqa` to work with argument `model_name_or_path` set to default value `'clip_iqa'`"
                ", package `piq` version v0.8.0 or later must be installed.") from err
        from transformers import CLIPProcessor

        return piq.clip_iqa.clip.load().eval(), CLIPProcessor.from_pretrained("openai/clip-vit-base-patch16")
    return _get_clip_model_and_processor(model_name_or_path)


def _clip_iqa_format_prompts(prompts: Tuple[Union[str, Tuple[str, str]]] = ("quality",)) -> Tuple[List[str], List[str]]:
    """(flat list of positive / negative prompts, prompt names)."""
    if not isinstance(prompts, tuple):
        raise ValueError("Argument `prompts` must be a tuple containing strings or tuples of strings")
    names: List[str] = []
    flat: List[str] = []
    count = 0
    for p in prompts:
        if not isinstance(p, (str, tuple)):
            raise ValueError("Argument `prompts` must be a tuple containing strings or tuples of strings")
        if isinstance(p, str):
            if p not in _PROMPTS:
                raise ValueError(
                    f"All elements of `prompts` must be one of {_PROMPTS.keys()} if not custom tuple prompts, got {p}.")
            names.append(p)
            flat.extend(_PROMPTS[p])
        else:
            if len(p) != 2:
                raise ValueError("If a tuple is provided in argument `prompts`, it must be of length 2")
            names.append(f"user_defined_{count}")
            flat.extend(p)
            count += 1
    return flat, names


def _clip_iqa_get_anchor_vectors(model_name_or_path: str, model, processor, prompts_list: List[str],
                                 device: Union[str, torch.device]) -> Tensor:
    if model_name_or_path == "clip_iqa":
        tp = processor(text=prompts_list)
        anchors_text = torch.zeros(len(prompts_list), processor.tokenizer.model_max_length, dtype=torch.long,
                                   device=device)
        for i, ids in enumerate(tp["input_ids"]):
            anchors_text[i, : len(ids)] = torch.tensor(ids, dtype=torch.long, device=device)
        anchors = model.encode_text(anchors_text).float()
    else:
        tp = processor(text=prompts_list, return_tensors="pt", padding=True)
        anchors = model.get_text_features(tp["input_ids"].to(device), tp["attention_mask"].to(device))
    return _normalize(anchors)


_CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
_CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def _clip_iqa_update(model_name_or_path: str, images: Tensor, model, processor, data_range: float,
                     device: Union[str, torch.device]) -> Tensor:
    images = images / float(data_range)
    if model_name_or_path == "clip_iqa":
        mean = torch.tensor(_CLIP_MEAN, device=device).view(1, 3, 1, 1)
        std = torch.tensor(_CLIP_STD, device=device).view(1, 3, 1, 1)
        feats = model.encode_image(((images - mean) / std).float(), pos_embedding=False).float()
    else:
        proc = processor(images=[i.cpu() for i in images], return_tensors="pt", padding=True)
        feats = model.get_image_features(proc["pixel_values"].to(device))
    return _normalize(feats)


def _clip_iqa_compute(img_features: Tensor, anchors: Tensor, prompts_names: List[str],
                      format_as_dict: bool = True) -> Union[Tensor, Dict[str, Tensor]]:
    """P(positive prompt) per image and prompt pair: softmax over each (positive, negative) logit pair."""
    if img_features.is_cuda and not (torch.is_grad_enabled() and img_features.requires_grad):
        # both dot products and the pair softmax in one launch (no [N, 2P] logits tensor)
        probs = ops.prompt_pair_prob(img_features, anchors, 100.0).to(img_features.dtype)
    else:
        logits = 100 * img_features @ anchors.t()
        probs = logits.reshape(logits.shape[0], -1, 2).softmax(-1)[:, :, 0]
    if len(prompts_names) == 1:
        return probs.squeeze()
    if format_as_dict:
        return {p: probs[:, i] for i, p in enumerate(prompts_names)}
    return probs


def clip_image_quality_assessment(images: Tensor, model_name_or_path: str = "clip_iqa", data_range: float = 1.0,
                                  prompts: Tuple[Union[str, Tuple[str, str]]] = ("quality",)
                                  ) -> Union[Tensor, Dict[str, Tensor]]:
    """CLIP-IQA probabilities per image (``F/multimodal/clip_iqa.py:196``)."""
    prompts_list, prompts_names = _clip_iqa_format_prompts(prompts)
    model, processor = _get_clip_iqa_model_and_processor(model_name_or_path)
    device = images.device
    model = model.to(device)
    with torch.inference_mode():
        anchors = _clip_iqa_get_anchor_vectors(model_name_or_path, model, processor, prompts_list, device)
        feats = _clip_iqa_update(model_name_or_path, images, model, processor, data_range, device)
        return _clip_iqa_compute(feats, anchors, prompts_names)


__all__ = ["clip_image_quality_assessment", "clip_score"]
