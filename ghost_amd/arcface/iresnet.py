"""Drop-in for ``arcface_model.iresnet`` (the ArcFace backbone GHOST loads as ``netArc``).

GHOST builds it as ``iresnet100(fp16=False)``, loads ``arcface_model/backbone.pth`` and calls it on
[N,3,112,112] crops in [-1, 1] (inference.py:33-36; core.py:43-54; video_processing.py:136-140).
The module file itself is a download (download_models.sh:3) that is absent from the reference
tree, so the definition here follows the public insightface ``arcface_torch`` IResNet: same
submodule names and state_dict keys (``conv1``, ``bn1``, ``prelu``, ``layerL.B.{bn1, conv1, bn2,
prelu, conv2, bn3, downsample.0, downsample.1}``, ``bn2``, ``fc``, ``features``), so a
``backbone.pth`` state_dict loads strictly.  Parity with the real module is unpinned (no source,
weights or fixtures available offline; see oracle/arcface_ref.py).

Execution: one call into libghost_amd.so (``ghost_arc_forward``) runs the network on the caller's
current HIP stream: implicit-GEMM convs on the matrix cores with BatchNorm/PReLU/residual fused into
their epilogues (arc_runtime.hip).  fp32 parameters run the fp32 path (the reference runs fp16=False);
``compute_dtype=torch.bfloat16`` runs bf16 storage with fp32 accumulation; embeddings are fp32 either
way.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch
import torch.nn as nn

from .. import _lib
from .._packed import PackedModule, WorkspaceCache

WIDTHS = (64, 128, 256, 512)


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation, groups=groups,
                     bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class IBasicBlock(nn.Module):
    """BN -> conv3x3 -> BN -> PReLU -> conv3x3/stride -> BN, + identity (downsample when reshaped)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1):
        super().__init__()
        if groups != 1 or base_width != 64 or dilation != 1:
            raise ValueError("IBasicBlock supports groups=1, base_width=64, dilation=1 only")
        self.bn1 = nn.BatchNorm2d(inplanes, eps=1e-05)
        self.conv1 = conv3x3(inplanes, planes)
        self.bn2 = nn.BatchNorm2d(planes, eps=1e-05)
        self.prelu = nn.PReLU(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn3 = nn.BatchNorm2d(planes, eps=1e-05)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        raise NotImplementedError("ghost_amd: IBasicBlock runs inside IResNet.forward on the MI355X path")


class _Runtime:
    def __init__(self, layers, nf, dtype, slots):
        self.lib = _lib.load()
        self.dtype = dtype
        h = C.c_void_p()
        arr = (C.c_int * 4)(*layers)
        _lib.check(self.lib.ghost_arc_create(arr, nf, _lib.gdtype(dtype), C.byref(h)), "ghost_arc_create")
        self.h = h
        self.slots = slots
        self.ws = WorkspaceCache()   # (N, stream) -> workspace
        for name, t in slots.items():
            _lib.check(self.lib.ghost_arc_bind(h, name.encode(), t.data_ptr(), t.numel()), f"bind {name}")
        if self.lib.ghost_arc_missing(h) != 0:
            _lib.check(-2, "ArcFace weights incomplete")

    def __del__(self):
        try:
            if self.h:
                self.lib.ghost_arc_destroy(self.h)
        except Exception:
            pass


class IResNet(PackedModule):
    fc_scale = 7 * 7

    def __init__(self, block, layers, dropout=0, num_features=512, zero_init_residual=False, groups=1,
                 width_per_group=64, replace_stride_with_dilation=None, fp16=False, *,
                 compute_dtype: Optional[torch.dtype] = None):
        super().__init__()
        if block is not IBasicBlock:
            raise ValueError("IResNet: only IBasicBlock is supported")
        if replace_stride_with_dilation not in (None, [False, False, False], (False, False, False)):
            raise ValueError("IResNet: dilation is not supported")
        self.fp16 = fp16
        self.compute_dtype = compute_dtype
        self.layers_cfg = tuple(int(n) for n in layers)
        self.num_features = num_features
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(self.inplanes, eps=1e-05)
        self.prelu = nn.PReLU(self.inplanes)
        for i, (w, n) in enumerate(zip(WIDTHS, layers), 1):
            setattr(self, f"layer{i}", self._make_layer(block, w, n, stride=2))
        self.bn2 = nn.BatchNorm2d(512 * block.expansion, eps=1e-05)
        self.dropout = nn.Dropout(p=dropout, inplace=True)
        self.fc = nn.Linear(512 * block.expansion * self.fc_scale, num_features)
        self.features = nn.BatchNorm1d(num_features, eps=1e-05)
        nn.init.constant_(self.features.weight, 1.0)
        self.features.weight.requires_grad = False
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.normal_(m.weight, 0, 0.1)
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, IBasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)
        self._init_packed()

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       nn.BatchNorm2d(planes * block.expansion, eps=1e-05))
        mods = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        mods += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    # -- weights ---------------------------------------------------------------------
    def _dtype(self):
        if self.compute_dtype is not None:
            return self.compute_dtype
        return torch.float32 if self.conv1.weight.dtype == torch.float32 else torch.bfloat16

    def _runtime(self, device):
        from .pack import pack_iresnet
        dt = self._dtype()
        return self._cached_runtime(device, dt, lambda sd: _Runtime(self.layers_cfg, self.num_features, dt,
                                                                     pack_iresnet(sd, self.layers_cfg, dt)))

    def _workspace(self, rt, N, dev):
        def nbytes():
            n = rt.lib.ghost_arc_workspace_bytes(rt.h, N)
            if n < 0:
                _lib.check(int(n), "ArcFace workspace sizing")
            return n
        return rt.ws.get((N, _lib.stream_ptr(dev)), nbytes, dev)

    # -- execution -------------------------------------------------------------------
    @torch.no_grad()
    def forward(self, x):
        """x: [N,3,112,112] (any strides, f32/f16/bf16) on the GPU -> fp32 [N, num_features]."""
        _lib.require_gpu(x, "IResNet.forward")
        if x.ndim != 4 or tuple(x.shape[1:]) != (3, 112, 112):
            raise RuntimeError(f"ghost_amd: IResNet expects [N,3,112,112], got {tuple(x.shape)}")
        if x.dtype not in (torch.float32, torch.float16, torch.bfloat16):
            raise TypeError(f"ghost_amd: unsupported input dtype {x.dtype}")
        rt = self._runtime(x.device)
        N = x.shape[0]
        emb = torch.empty(N, self.num_features, dtype=torch.float32, device=x.device)
        ws = self._workspace(rt, N, x.device)
        st = (C.c_int64 * 4)(*x.stride())
        _lib.check(rt.lib.ghost_arc_forward(rt.h, x.data_ptr(), _lib.gdtype(x.dtype), st, N, emb.data_ptr(),
                                            ws.data_ptr(), ws.numel(), _lib.stream_ptr(x.device)), "IResNet.forward")
        return emb

    @torch.no_grad()
    def forward_taps(self, x):
        """forward + every stage's stored tensors (parity bisection against the storage-emulating oracle):
        a list over stages (0 = stem, i = IBasicBlock i) of (X_i, BN(X_i)) as NCHW views in the compute
        dtype — X_i the residual stream, BN(X_i) the next BatchNorm's output the next conv reads."""
        _lib.require_gpu(x, "IResNet.forward_taps")
        rt = self._runtime(x.device)
        N, dev = x.shape[0], x.device
        shapes = [(112, 64)]
        for planes, n in zip((64, 128, 256, 512), self.layers_cfg):
            for b in range(n):
                shapes.append((shapes[-1][0] // (2 if b == 0 else 1), planes))
        bufs = [(torch.empty(N, h, h, c, dtype=rt.dtype, device=dev), torch.empty(N, h, h, c, dtype=rt.dtype, device=dev))
                for h, c in shapes]
        ptrs = (C.c_void_p * (2 * len(bufs)))(*[t.data_ptr() for pair in bufs for t in pair])
        _lib.check(rt.lib.ghost_arc_set_taps(rt.h, ptrs, 2 * len(bufs)), "arc taps")
        try:
            emb = self.forward(x)
        finally:
            rt.lib.ghost_arc_set_taps(rt.h, None, 0)
        return emb, [(a.permute(0, 3, 1, 2), b.permute(0, 3, 1, 2)) for a, b in bufs]

    @torch.no_grad()
    def embed_u8(self, crops: torch.Tensor) -> torch.Tensor:
        """Fused netArc(F.interpolate(normalize_and_torch_batch(crops), 0.5, bilinear, align_corners=True))
        on device uint8 crops [N,224,224,3] (video_processing.py:136-139, core.py:43-44)."""
        _lib.require_gpu(crops, "IResNet.embed_u8")
        if crops.dtype != torch.uint8 or crops.ndim != 4 or crops.shape[3] != 3:
            raise RuntimeError("ghost_amd: crops must be uint8 [N,H,W,3]")
        if crops[0].stride() != (crops.shape[2] * 3, 3, 1):
            crops = crops.contiguous()
        rt = self._runtime(crops.device)
        N, H, W = crops.shape[:3]
        emb = torch.empty(N, self.num_features, dtype=torch.float32, device=crops.device)
        ws = self._workspace(rt, N, crops.device)
        _lib.check(rt.lib.ghost_arc_embed_u8(rt.h, crops.data_ptr(), crops.stride(0), N, H, W, emb.data_ptr(),
                                             ws.data_ptr(), ws.numel(), _lib.stream_ptr(crops.device)),
                   "IResNet.embed_u8")
        return emb


def _iresnet(arch, block, layers, pretrained, progress, **kwargs):
    if pretrained:
        raise ValueError("ghost_amd: no pretrained download offline; load backbone.pth with load_state_dict")
    return IResNet(block, layers, **kwargs)


def iresnet18(pretrained=False, progress=True, **kwargs):
    return _iresnet('iresnet18', IBasicBlock, [2, 2, 2, 2], pretrained, progress, **kwargs)


def iresnet34(pretrained=False, progress=True, **kwargs):
    return _iresnet('iresnet34', IBasicBlock, [3, 4, 6, 3], pretrained, progress, **kwargs)


def iresnet50(pretrained=False, progress=True, **kwargs):
    return _iresnet('iresnet50', IBasicBlock, [3, 4, 14, 3], pretrained, progress, **kwargs)


def iresnet100(pretrained=False, progress=True, **kwargs):
    return _iresnet('iresnet100', IBasicBlock, [3, 13, 30, 3], pretrained, progress, **kwargs)
