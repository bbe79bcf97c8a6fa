"""ORACLE — CPU restatement of the ArcFace identity encoder GHOST calls (test infrastructure only).

Imported only by ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg; the product
(``ghost_amd.arcface``) never imports or calls it.

PARITY UNPINNED.  GHOST loads ``arcface_model.iresnet.iresnet100`` (inference.py:15,33-36;
train-upsampler.py:26,261-264; export-onnx.py:4,56-57), but ``arcface_model/iresnet.py`` is not in
the reference tree: ``download_models.sh:3`` fetches it, together with its weights, from a GitHub
release.  Neither the definition nor the weights exist in this container, and the reference holds
no test or fixture for it.  This file restates the public insightface ``arcface_torch`` IResNet
(the module that download ships), from its published design:

* ``IBasicBlock``: BN -> conv3x3/s1 -> BN -> PReLU -> conv3x3/stride -> BN, + identity
  (identity = conv1x1/stride + BN when the shape changes), no activation after the sum;
* ``IResNet``: conv3x3 3->64 /s1 -> BN -> PReLU; layers of widths 64/128/256/512, each opened by a
  stride-2 block; BN2d -> flatten (NCHW order) -> dropout (identity in eval) -> Linear(512*7*7 ->
  512) -> BatchNorm1d ("features"); BN eps 1e-5;
* depths: iresnet18 [2,2,2,2], iresnet34 [3,4,6,3], iresnet50 [3,4,14,3], iresnet100 [3,13,30,3].

Only self-consistency (the HIP path against this restatement) can be checked; it is called
"parity unpinned" in DESIGN.md and in the tests.

The pipeline arithmetic around it IS in the reference and is restated from there:
* ``normalize_and_torch_batch`` (utils/inference/image_processing.py:37-48): u8 NHWC (BGR, no
  channel swap) -> /255 only if the batch max > 1 -> NCHW -> (x - 0.5)/0.5;
* ``F.interpolate(scale_factor=0.5, mode='bilinear', align_corners=True)`` (core.py:44,53;
  video_processing.py:138): 224 -> 112;
* face matching (video_processing.py:126,139-148): F.normalize both sides, similarity =
  faces @ targets.T, best face per target = argmax over faces, accepted if > similarity_th.
"""
from __future__ import annotations

import zlib
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5
LAYERS = {"iresnet18": [2, 2, 2, 2], "iresnet34": [3, 4, 6, 3], "iresnet50": [3, 4, 14, 3],
          "iresnet100": [3, 13, 30, 3]}
WIDTHS = [64, 128, 256, 512]


def blocks(layers) -> List[Tuple[int, int, int, int, int]]:
    """(layer, block, inplanes, planes, stride) in forward order; each layer opens with stride 2."""
    out, inplanes = [], 64
    for li, (planes, n) in enumerate(zip(WIDTHS, layers), 1):
        for b in range(n):
            out.append((li, b, inplanes, planes, 2 if b == 0 else 1))
            inplanes = planes
    return out


def param_specs(layers=LAYERS["iresnet100"], num_features: int = 512):
    """Ordered (key, shape, kind) of the arcface_torch IResNet state_dict."""
    specs: List[Tuple[str, Tuple[int, ...], str]] = []

    def bn(prefix, c):
        specs.extend([(f"{prefix}.weight", (c,), "bn_w"), (f"{prefix}.bias", (c,), "bn_b"),
                      (f"{prefix}.running_mean", (c,), "bn_rm"), (f"{prefix}.running_var", (c,), "bn_rv"),
                      (f"{prefix}.num_batches_tracked", (), "bn_nbt")])

    specs.append(("conv1.weight", (64, 3, 3, 3), "conv"))
    bn("bn1", 64)
    specs.append(("prelu.weight", (64,), "prelu"))
    for li, b, inp, planes, stride in blocks(layers):
        pre = f"layer{li}.{b}"
        bn(f"{pre}.bn1", inp)
        specs.append((f"{pre}.conv1.weight", (planes, inp, 3, 3), "conv"))
        bn(f"{pre}.bn2", planes)
        specs.append((f"{pre}.prelu.weight", (planes,), "prelu"))
        specs.append((f"{pre}.conv2.weight", (planes, planes, 3, 3), "conv"))
        bn(f"{pre}.bn3", planes)
        if b == 0:
            specs.append((f"{pre}.downsample.0.weight", (planes, inp, 1, 1), "conv"))
            bn(f"{pre}.downsample.1", planes)
    bn("bn2", 512)
    specs.append(("fc.weight", (num_features, 512 * 49), "fc_w"))
    specs.append(("fc.bias", (num_features,), "bias"))
    bn("features", num_features)
    return specs


def make_weights(specs, dtype=torch.float32) -> Dict[str, torch.Tensor]:
    """Deterministic key-hashed synthetic weights (no checkpoint offline): He-normal convs (keeps the
    100-block residual stream bounded with BN gamma ~ U(0.5, 1)), PReLU slopes U(0.1, 0.3), fc
    N(0, 1/sqrt(fan_in))."""
    out: Dict[str, torch.Tensor] = {}
    for key, shape, kind in specs:
        if kind == "bn_nbt":
            out[key] = torch.zeros((), dtype=torch.int64)
            continue
        g = np.random.Generator(np.random.PCG64(zlib.crc32(("arc." + key).encode())))
        if kind == "conv":
            fan_in = int(np.prod(shape[1:]))
            a = g.normal(0.0, np.sqrt(1.0 / fan_in), size=shape)
        elif kind == "fc_w":
            a = g.normal(0.0, 1.0 / np.sqrt(shape[1]), size=shape)
        elif kind == "bias":
            a = g.normal(0.0, 0.02, size=shape)
        elif kind == "prelu":
            a = g.uniform(0.1, 0.3, size=shape)
        elif kind == "bn_w":
            a = g.uniform(0.5, 1.0, size=shape)
        elif kind == "bn_rv":
            a = g.uniform(0.5, 1.5, size=shape)
        elif kind in ("bn_b", "bn_rm"):
            a = g.normal(0.0, 0.1, size=shape)
        else:  # pragma: no cover
            raise ValueError(kind)
        out[key] = torch.from_numpy(np.asarray(a, dtype=np.float32)).to(dtype)
    return out


def _bn(x, p, prefix):
    return F.batch_norm(x, p[f"{prefix}.running_mean"].to(x.dtype), p[f"{prefix}.running_var"].to(x.dtype),
                        p[f"{prefix}.weight"].to(x.dtype), p[f"{prefix}.bias"].to(x.dtype), False, 0.0, BN_EPS)


@torch.no_grad()
def iresnet_forward(p, x, layers=LAYERS["iresnet100"]):
    """IResNet.forward in eval mode: x [N,3,112,112] -> [N, num_features]."""
    dt = x.dtype
    x = F.prelu(_bn(F.conv2d(x, p["conv1.weight"].to(dt), None, padding=1), p, "bn1"), p["prelu.weight"].to(dt))
    for li, b, _inp, _planes, stride in blocks(layers):
        pre = f"layer{li}.{b}"
        out = _bn(x, p, f"{pre}.bn1")
        out = F.conv2d(out, p[f"{pre}.conv1.weight"].to(dt), None, padding=1)
        out = F.prelu(_bn(out, p, f"{pre}.bn2"), p[f"{pre}.prelu.weight"].to(dt))
        out = _bn(F.conv2d(out, p[f"{pre}.conv2.weight"].to(dt), None, stride=stride, padding=1), p, f"{pre}.bn3")
        idn = x
        if b == 0:
            idn = _bn(F.conv2d(x, p[f"{pre}.downsample.0.weight"].to(dt), None, stride=stride), p,
                      f"{pre}.downsample.1")
        x = out + idn
    x = _bn(x, p, "bn2")
    x = torch.flatten(x, 1)
    x = F.linear(x, p["fc.weight"].to(dt), p["fc.bias"].to(dt))
    return F.batch_norm(x, p["features.running_mean"].to(dt), p["features.running_var"].to(dt),
                        p["features.weight"].to(dt), p["features.bias"].to(dt), False, 0.0, BN_EPS)


# ----------------------------------------------------------------------------------------------------
# bf16-storage emulation of the runtime's plan (arc_runtime.hip): the same network with every tensor the
# runtime stores rounded to bf16 where it stores it, fp32 in between:
#   input x (after the prep kernel)                   -> bf16
#   conv weights (stem, conv1/conv2, downsample, fc)  -> bf16 (BatchNorms stay fp32 epilogue scale/shift)
#   stem  v = PReLU(bn1(conv(x)));         X = q(v), XB = q(bn1_block1(v))
#   block T = q(PReLU(bn2(conv1(XB))));    R = q(bn(down(X))) (first block of a layer);
#         v = bn3(conv2/s(T)) + (R | X);   X' = q(v), XB' = q(next BN(v))  (the head's bn2 after the last)
#   head  emb = features(fc(flatten(XB))) in fp32 (bf16 operands)
# ----------------------------------------------------------------------------------------------------
def _qs(t, store):
    return t.to(store).float()


def stem_storage(p, x, store=torch.bfloat16, first_bn="layer1.0.bn1"):
    """Stage 0 from the stored input x: (X, XB)."""
    v = F.prelu(_bn(F.conv2d(x, _qs(p["conv1.weight"].float(), store), None, padding=1), p, "bn1"),
                p["prelu.weight"].float())
    return _qs(v, store), _qs(_bn(v, p, first_bn), store)


def block_storage(p, X, XB, li, b, stride, next_bn, store=torch.bfloat16):
    """IBasicBlock (li, b) from the stored (X, XB) of the stage before it: its stored (X', XB')."""
    pre = f"layer{li}.{b}"
    wq = lambda k: _qs(p[k].float(), store)  # noqa: E731
    t = F.conv2d(XB, wq(f"{pre}.conv1.weight"), None, padding=1)
    T = _qs(F.prelu(_bn(t, p, f"{pre}.bn2"), p[f"{pre}.prelu.weight"].float()), store)
    res = X
    if b == 0:
        res = _qs(_bn(F.conv2d(X, wq(f"{pre}.downsample.0.weight"), None, stride=stride), p, f"{pre}.downsample.1"),
                  store)
    v = _bn(F.conv2d(T, wq(f"{pre}.conv2.weight"), None, stride=stride, padding=1), p, f"{pre}.bn3") + res
    return _qs(v, store), _qs(_bn(v, p, next_bn), store)


def head_storage(p, XB, store=torch.bfloat16):
    x = F.linear(torch.flatten(XB, 1), _qs(p["fc.weight"].float(), store), p["fc.bias"].float())
    return F.batch_norm(x, p["features.running_mean"].float(), p["features.running_var"].float(),
                        p["features.weight"].float(), p["features.bias"].float(), False, 0.0, BN_EPS)


def next_bn_names(layers):
    """The BatchNorm each stage's second output applies: the next block's bn1, the head's bn2 last."""
    bl = blocks(layers)
    return [f"layer{li}.{b}.bn1" for li, b, *_ in bl] + ["bn2"]


@torch.no_grad()
def iresnet_forward_storage(p, x, layers=LAYERS["iresnet100"], store=torch.bfloat16):
    """The runtime's bf16 plan end to end -> (emb, [(X_i, XB_i)] per stage)."""
    nb = next_bn_names(layers)
    x = _qs(x.float(), store)
    X, XB = stem_storage(p, x, store, nb[0])
    stages = [(X, XB)]
    for i, (li, b, _inp, _planes, stride) in enumerate(blocks(layers)):
        X, XB = block_storage(p, X, XB, li, b, stride, nb[i + 1], store)
        stages.append((X, XB))
    return head_storage(p, XB, store), stages


def normalize_batch_u8(frames_u8: np.ndarray) -> torch.Tensor:
    """normalize_and_torch_batch (image_processing.py:37-48) on CPU: u8 NHWC -> NCHW in [-1, 1]."""
    t = torch.from_numpy(frames_u8.copy())
    if t.max() > 1.:
        t = t / 255.
    t = t.permute(0, 3, 1, 2)
    return (t - 0.5) / 0.5


def preprocess_crops(frames_u8: np.ndarray) -> torch.Tensor:
    """F.interpolate(normalize_and_torch_batch(crops), scale_factor=0.5, bilinear, align_corners=True)
    (core.py:43-44, video_processing.py:137-139): the network input."""
    x = normalize_batch_u8(frames_u8).float()
    return F.interpolate(x, scale_factor=0.5, mode="bilinear", align_corners=True)


def embed_crops(p, frames_u8: np.ndarray, layers=LAYERS["iresnet100"]) -> torch.Tensor:
    """netArc(preprocess_crops(crops))."""
    return iresnet_forward(p, preprocess_crops(frames_u8), layers)


def match_faces(face_embeds: torch.Tensor, target_embeds: torch.Tensor, similarity_th: float):
    """video_processing.py:126,140-148: per target, the most similar face and whether it passes the threshold."""
    t = F.normalize(target_embeds)
    f = F.normalize(face_embeds)
    sim = f @ t.T
    best = sim.argmax(0)
    ok = torch.stack([sim[best[j], j] > similarity_th for j in range(t.shape[0])])
    return best, sim[best, torch.arange(t.shape[0])], ok


def make_u8_faces(n: int, size: int = 224, seed: int = 3) -> np.ndarray:
    """Synthetic aligned face crops u8 [n, size, size, 3] (smooth random fields: natural-image-like
    low-frequency content, so the 0.5x resize is exercised on non-white-noise input)."""
    g = np.random.Generator(np.random.PCG64(seed))
    lo = g.uniform(0, 255, size=(n, size // 16, size // 16, 3)).astype(np.float32)
    t = torch.from_numpy(lo).permute(0, 3, 1, 2)
    up = F.interpolate(t, size=(size, size), mode="bilinear", align_corners=False).permute(0, 2, 3, 1).numpy()
    noise = g.normal(0, 8, size=up.shape)
    return np.clip(up + noise, 0, 255).astype(np.uint8)
