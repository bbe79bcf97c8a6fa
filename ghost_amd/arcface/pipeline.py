"""The ArcFace calls of GHOST's inference pipeline, on the device.

* ``normalize_and_torch_batch`` — utils/inference/image_processing.py:37-48 (same semantics:
  divide by 255 only when the batch max exceeds 1; channel order kept);
* ``embed_crops`` — ``netArc(F.interpolate(normalize_and_torch_batch(crops), scale_factor=0.5,
  mode='bilinear', align_corners=True))`` (core.py:43-44, video_processing.py:136-139), fused into
  one native call (``ghost_arc_embed_u8``);
* ``match_faces`` — the per-frame identity matching of video_processing.py:126,139-148
  (``ghost_arc_match``).
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple

import numpy as np
import torch

from .. import _lib


def normalize_and_torch_batch(frames, device="cuda") -> torch.Tensor:
    """u8 NHWC frames (numpy or tensor) -> [N,3,H,W] in [-1,1] on the device (image_processing.py:37-48)."""
    t = torch.as_tensor(np.ascontiguousarray(frames) if isinstance(frames, np.ndarray) else frames).to(device)
    _lib.require_gpu(t, "normalize_and_torch_batch")
    if t.max() > 1.:
        t = t / 255.
    t = t.permute(0, 3, 1, 2)
    return (t - 0.5) / 0.5


def embed_crops(net, crops) -> torch.Tensor:
    """Embeddings of uint8 aligned crops [N,224,224,3] (numpy or device tensor) with the fused native path."""
    if isinstance(crops, np.ndarray):
        crops = torch.from_numpy(np.ascontiguousarray(crops)).cuda()
    return net.embed_u8(crops)


def match_faces(face_embeds: torch.Tensor, target_embeds: torch.Tensor,
                similarity_th: float = 0.15) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Per target: (index of the most similar face, its cosine similarity, accepted = sim > th)."""
    _lib.require_gpu(face_embeds, "match_faces")
    f = face_embeds.float().contiguous()
    t = target_embeds.float().contiguous()
    if f.ndim != 2 or t.ndim != 2 or f.shape[1] != t.shape[1]:
        raise RuntimeError("ghost_amd: match_faces expects [F, D] and [T, D] embeddings")
    T = t.shape[0]
    best = torch.empty(T, dtype=torch.int32, device=f.device)
    sim = torch.empty(T, dtype=torch.float32, device=f.device)
    ok = torch.empty(T, dtype=torch.int32, device=f.device)
    lib = _lib.load()
    _lib.check(lib.ghost_arc_match(f.data_ptr(), f.shape[0], t.data_ptr(), T, f.shape[1], C.c_float(similarity_th),
                                   best.data_ptr(), sim.data_ptr(), ok.data_ptr(), _lib.stream_ptr(f.device)),
               "match_faces")
    return best.long(), sim, ok.bool()
