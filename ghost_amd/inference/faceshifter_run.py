"""faceshifter_batch (utils/inference/faceshifter_run.py:5-22) on the MI355X path.

The tanh -> ((Y*0.5+0.5)*255)[..., BGR] -> uint8 post-processing is fused into the
epilogue of the generator's last conv (no extra pass over Y); the identity row is
broadcast by a zero row stride instead of ``torch.cat([source_emb]*bs)``.
"""
from __future__ import annotations

import numpy as np
import torch


def faceshifter_batch(source_emb: torch.Tensor, target: torch.Tensor, G: torch.nn.Module) -> np.ndarray:
    """Apply the swap network to a batch of target crops; returns uint8 BGR [B,256,256,3] on the host."""
    bs = target.shape[0]
    assert target.ndim == 4, "target should have 4 dimentions -- B x C x H x W"
    z = source_emb.reshape(source_emb.shape[0], -1)
    if bs > 1 and z.shape[0] == 1:
        z = z.expand(bs, -1)          # faceshifter_run.py:15-16, without materialising the copies
    out = torch.empty(bs, 256, 256, 3, dtype=torch.uint8, device=target.device)
    with torch.no_grad():
        G(target, z, out_u8=out)
    return out.cpu().numpy()


def faceshifter_batch_u8(source_emb: torch.Tensor, crops_u8: torch.Tensor, G: torch.nn.Module,
                         out: torch.Tensor = None) -> torch.Tensor:
    """Fully fused variant: device uint8 BGR crops in, device uint8 BGR swaps out (stays in HBM)."""
    return G.swap_u8(crops_u8, source_emb, out=out)
