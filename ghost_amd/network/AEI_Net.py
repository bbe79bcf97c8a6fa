"""Drop-in for network/AEI_Net.py on MI355X.

``AEI_Net(backbone, num_blocks=2, c_id=256)`` keeps the reference constructor,
submodule names and state_dict keys (AEI_Net.py:19-159), so
``G.load_state_dict(torch.load(path, map_location='cpu'))``, ``.cuda()``, ``.half()``,
``.eval()`` and ``forward(Xt, z_id) -> (Y, attr)`` / ``get_attr(X)`` behave as in
inference.py:26-30 and faceshifter_run.py:19.

Execution: the whole forward is one call into libghost_amd.so (``ghost_aei_forward``),
which runs hand-written gfx950 kernels on the caller's current HIP stream.  The weights
are packed once per (device, dtype) into the kernels' layouts (pack.py) and re-packed
automatically when a parameter changes.  Outputs are NHWC in device memory; ``Y`` and
the attr maps are returned as NCHW *views* (``channels_last`` strides) — same shapes and
values as the reference, no copy.

Numerics: fp32 parameters run the fp32 path (exact-fp32 MFMA, |dY| <= 1e-3 vs the
reference CPU forward).  ``.bfloat16()`` parameters (or ``compute_dtype=torch.bfloat16``)
run the bf16 throughput path (bf16 storage, fp32 accumulation) and return bf16 tensors.
``.half()`` parameters (inference.py:30; or ``compute_dtype=torch.float16``) run the same
kernels instantiated for fp16 storage (v_mfma_f32_16x16x32_f16, fp32 accumulation) and
return float16 tensors: the reference's own GPU precision, ~4x more accurate end to end than
bf16 storage.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch
import torch.nn as nn

from .. import _lib
from .._packed import PackedModule, WorkspaceCache
from .AADLayer import AAD_ResBlk, AADLayer, AddBlocksSequential  # noqa: F401  (reference re-exports)
from .pack import pack_all
from .resnet import MLAttrEncoderResnet


def weight_init(m):
    """AEI_Net.py:8-16 (irrelevant once a checkpoint is loaded; kept for state parity)."""
    if isinstance(m, nn.Linear):
        m.weight.data.normal_(0, 0.001)
        m.bias.data.zero_()
    if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
        nn.init.xavier_normal_(m.weight.data)


class _Container(nn.Sequential):
    def forward(self, *inputs):
        raise NotImplementedError("ghost_amd: encoder blocks run inside AEI_Net.forward / get_attr on the MI355X path")


def conv4x4(in_c, out_c, norm=nn.BatchNorm2d):
    """Conv4x4/s2/p1 -> BN -> LeakyReLU(0.1) container (AEI_Net.py:19-24)."""
    return _Container(nn.Conv2d(in_channels=in_c, out_channels=out_c, kernel_size=4, stride=2, padding=1, bias=False),
                      norm(out_c), nn.LeakyReLU(0.1, inplace=True))


class deconv4x4(nn.Module):
    """ConvT4x4/s2/p1 -> BN -> LReLU -> cat / add skip (AEI_Net.py:27-41)."""

    def __init__(self, in_c, out_c, norm=nn.BatchNorm2d):
        super().__init__()
        self.deconv = nn.ConvTranspose2d(in_channels=in_c, out_channels=out_c, kernel_size=4, stride=2, padding=1,
                                         bias=False)
        self.bn = norm(out_c)
        self.lrelu = nn.LeakyReLU(0.1, inplace=True)

    def forward(self, input, skip, backbone):
        raise NotImplementedError("ghost_amd: deconv4x4 runs inside AEI_Net.forward / get_attr on the MI355X path")


class MLAttrEncoder(nn.Module):
    """Multi-level attribute encoder (AEI_Net.py:44-95)."""

    def __init__(self, backbone):
        super().__init__()
        self.backbone = backbone
        self.conv1 = conv4x4(3, 32)
        self.conv2 = conv4x4(32, 64)
        self.conv3 = conv4x4(64, 128)
        self.conv4 = conv4x4(128, 256)
        self.conv5 = conv4x4(256, 512)
        self.conv6 = conv4x4(512, 1024)
        self.conv7 = conv4x4(1024, 1024)
        if backbone == 'unet':
            chans = [(1024, 1024), (2048, 512), (1024, 256), (512, 128), (256, 64), (128, 32)]
        elif backbone == 'linknet':
            chans = [(1024, 1024), (1024, 512), (512, 256), (256, 128), (128, 64), (64, 32)]
        else:
            chans = []
        for i, (ci, co) in enumerate(chans, 1):
            setattr(self, f"deconv{i}", deconv4x4(ci, co))
        self.apply(weight_init)
        self._owner = None

    def forward(self, Xt):
        if self._owner is None:
            raise NotImplementedError("ghost_amd: call AEI_Net.get_attr (the encoder runs as part of the AEI_Net plan)")
        return self._owner().get_attr(Xt)


class AADGenerator(nn.Module):
    """AAD generator (AEI_Net.py:98-139); executed by AEI_Net.forward."""

    def __init__(self, backbone, c_id=256, num_blocks=2):
        super().__init__()
        self.up1 = nn.ConvTranspose2d(c_id, 1024, kernel_size=2, stride=1, padding=0)
        self.AADBlk1 = AAD_ResBlk(1024, 1024, 1024, c_id, num_blocks)
        if backbone == 'linknet':
            self.AADBlk2 = AAD_ResBlk(1024, 1024, 1024, c_id, num_blocks)
            self.AADBlk3 = AAD_ResBlk(1024, 1024, 512, c_id, num_blocks)
            self.AADBlk4 = AAD_ResBlk(1024, 512, 256, c_id, num_blocks)
            self.AADBlk5 = AAD_ResBlk(512, 256, 128, c_id, num_blocks)
            self.AADBlk6 = AAD_ResBlk(256, 128, 64, c_id, num_blocks)
            self.AADBlk7 = AAD_ResBlk(128, 64, 32, c_id, num_blocks)
            self.AADBlk8 = AAD_ResBlk(64, 3, 32, c_id, num_blocks)
        else:
            self.AADBlk2 = AAD_ResBlk(1024, 1024, 2048, c_id, num_blocks)
            self.AADBlk3 = AAD_ResBlk(1024, 1024, 1024, c_id, num_blocks)
            self.AADBlk4 = AAD_ResBlk(1024, 512, 512, c_id, num_blocks)
            self.AADBlk5 = AAD_ResBlk(512, 256, 256, c_id, num_blocks)
            self.AADBlk6 = AAD_ResBlk(256, 128, 128, c_id, num_blocks)
            self.AADBlk7 = AAD_ResBlk(128, 64, 64, c_id, num_blocks)
            self.AADBlk8 = AAD_ResBlk(64, 3, 64, c_id, num_blocks)
        self.apply(weight_init)

    def forward(self, z_attr, z_id):
        raise NotImplementedError("ghost_amd: AADGenerator runs inside AEI_Net.forward on the MI355X path")


# per-handle plan options (include/ghost_amd.h GHOST_AEI_OPT_*)
OPTIONS = {"fuse_upsample": 0, "fuse_stats": 1, "two_streams": 2, "tap_partials": 3, "fuse_reduce": 4}


class _Runtime:
    """Native handle + packed weights for one (device, compute dtype)."""

    def __init__(self, backbone, num_blocks, c_id, dtype, slots, options=None):
        self.lib = _lib.load()
        self.dtype = dtype
        h = C.c_void_p()
        _lib.check(self.lib.ghost_aei_create(backbone.encode(), num_blocks, c_id, _lib.gdtype(dtype), C.byref(h)),
                   "ghost_aei_create")
        self.h = h
        self.slots = slots  # keeps the packed tensors alive
        for name, t in slots.items():
            _lib.check(self.lib.ghost_aei_bind(h, name.encode(), t.data_ptr(), t.numel()), f"bind {name}")
        if self.lib.ghost_aei_missing(h) != 0:
            _lib.check(-2, "weights incomplete")
        for name, v in (options or {}).items():
            _lib.check(self.lib.ghost_aei_set_option(h, OPTIONS[name], int(v)), f"option {name}")
        self.ws = WorkspaceCache()   # (mode, B, stream) -> workspace (stream-ordered reuse)
        self.geom = []
        for k in range(1, 9):
            c_, h_, w_ = C.c_int(), C.c_int(), C.c_int()
            _lib.check(self.lib.ghost_aei_attr_geometry(h, k, C.byref(c_), C.byref(h_), C.byref(w_)))
            self.geom.append((c_.value, h_.value, w_.value))

    def workspace(self, mode: str, B: int, dev: torch.device, stream: int) -> torch.Tensor:
        fn = {"swap": self.lib.ghost_aei_swap_workspace_bytes,
              "idtable": self.lib.ghost_aei_identity_table_workspace_bytes}.get(mode, self.lib.ghost_aei_workspace_bytes)

        def nbytes():
            n = fn(self.h, B)
            if n < 0:
                _lib.check(int(n), "workspace sizing")
            return n
        return self.ws.get((mode, B, stream), nbytes, dev)

    def __del__(self):
        try:
            if self.h:
                self.lib.ghost_aei_destroy(self.h)
        except Exception:
            pass


class IdentityTable:
    """Device rows of ``AEI_Net.identity_table``: per source identity, every AADLayer's gamma_id / beta_id (fp32) and
    up1's output (the plan dtype).  Holds the runtime (packed weights, handle) it was computed with, so a table from
    before a re-pack is detected instead of used."""

    def __init__(self, rt, buf: torch.Tensor, off: int, n: int, device: torch.device):
        self.rt, self.buf, self.n, self.device = rt, buf, n, device
        self.ptr = buf.data_ptr() + off
        self.nbytes = buf.numel() - off       # what the native swap checks against the size n rows need

    def __len__(self):
        return self.n


class AEI_Net(PackedModule):
    """AEI_Net(backbone, num_blocks=2, c_id=256)  (AEI_Net.py:143-159)."""

    def __init__(self, backbone, num_blocks=2, c_id=256, *, compute_dtype: Optional[torch.dtype] = None):
        super().__init__()
        self.c_id = c_id
        self.backbone = backbone
        self.num_blocks = num_blocks
        self.compute_dtype = compute_dtype
        if backbone in ['unet', 'linknet']:
            self.encoder = MLAttrEncoder(backbone)
        elif backbone == 'resnet':
            self.encoder = MLAttrEncoderResnet()
        else:
            raise ValueError(f"unknown backbone {backbone!r}")
        self.generator = AADGenerator(backbone, c_id, num_blocks)
        self._options = {}
        import weakref
        self.encoder._owner = weakref.ref(self)
        self._init_packed()

    # -- weights -------------------------------------------------------------------
    def _dtype(self) -> torch.dtype:
        """Storage dtype of the plan: compute_dtype if given, else the parameters' (fp32, bf16 or fp16)."""
        if self.compute_dtype is not None:
            if self.compute_dtype not in (torch.float32, torch.bfloat16, torch.float16):
                raise TypeError(f"ghost_amd: unsupported compute_dtype {self.compute_dtype}")
            return self.compute_dtype
        dt = self.generator.up1.weight.dtype
        return dt if dt in (torch.float32, torch.float16) else torch.bfloat16

    def _out_dtype(self, rt) -> torch.dtype:
        """The dtype of the returned tensors: the plan's storage dtype."""
        return rt.dtype

    def set_option(self, name: str, value: int) -> None:
        """Per-model plan option (include/ghost_amd.h): fuse_upsample, fuse_stats, two_streams (0 / 1),
        tap_partials (0 / 1 / 2)."""
        if name not in OPTIONS:
            raise ValueError(f"ghost_amd: unknown option {name!r} (known: {sorted(OPTIONS)})")
        self._options[name] = int(value)
        if self._rt is not None:
            _lib.check(self._rt.lib.ghost_aei_set_option(self._rt.h, OPTIONS[name], int(value)), f"option {name}")
            self._rt.ws.clear()   # the plan (and so its workspace size) depends on the options

    def get_option(self, name: str) -> int:
        """The plan option's value in effect (the handle's, once a forward has created it)."""
        if name not in OPTIONS:
            raise ValueError(f"ghost_amd: unknown option {name!r} (known: {sorted(OPTIONS)})")
        if self._rt is not None:
            v = C.c_int()
            _lib.check(self._rt.lib.ghost_aei_get_option(self._rt.h, OPTIONS[name], C.byref(v)), f"option {name}")
            return int(v.value)
        if name in self._options:
            return self._options[name]
        raise RuntimeError("ghost_amd: option defaults live in the native handle; run a forward first")

    def _runtime(self, device) -> _Runtime:
        """The packed runtime for (device, dtype) (_packed.PackedModule: re-packed after load_state_dict,
        .to/.half, or an in-place change of any parameter or buffer)."""
        dt = self._dtype()
        return self._cached_runtime(device, dt, lambda sd: _Runtime(
            self.backbone, self.num_blocks, self.c_id, dt, pack_all(sd, self.backbone, self.num_blocks, self.c_id, dt),
            self._options))

    # -- execution -----------------------------------------------------------------
    def _prep(self, Xt, what):
        _lib.require_gpu(Xt, what)
        if Xt.ndim != 4 or tuple(Xt.shape[1:]) != (3, 256, 256):
            raise RuntimeError(f"ghost_amd: {what} expects Xt of shape [B,3,256,256], got {tuple(Xt.shape)}")
        if Xt.dtype not in (torch.float32, torch.float16, torch.bfloat16):
            raise TypeError(f"ghost_amd: unsupported input dtype {Xt.dtype}")
        rt = self._runtime(Xt.device)
        B = Xt.shape[0]
        attrs = [torch.empty(B, h, w, c, dtype=rt.dtype, device=Xt.device) for (c, h, w) in rt.geom]
        st = (C.c_int64 * 4)(*Xt.stride())
        return rt, B, attrs, st

    @torch.no_grad()
    def forward(self, Xt, z_id, *, out_u8: Optional[torch.Tensor] = None):
        Y, attrs, _ = self._forward(Xt, z_id, out_u8, taps=False)
        return Y, attrs

    @torch.no_grad()
    def forward_taps(self, Xt, z_id, *, out_u8: Optional[torch.Tensor] = None):
        """forward + the stored outputs of AADBlk1..7 (NCHW views, before the x2 upsample): the
        per-stage checkpoints the bf16 parity tests bisect against the storage-emulating oracle."""
        return self._forward(Xt, z_id, out_u8, taps=True)

    def _forward(self, Xt, z_id, out_u8, taps):
        rt, B, attrs, st = self._prep(Xt, "AEI_Net.forward")
        _lib.require_same_device(z_id, Xt.device, "z_id")
        z = z_id.reshape(z_id.shape[0], -1)
        if z.shape[0] != B or z.shape[1] != self.c_id:
            raise RuntimeError(f"ghost_amd: z_id must hold {B} rows of {self.c_id}, got {tuple(z_id.shape)}")
        if z.stride(1) != 1:
            z = z.contiguous()
        dev = Xt.device
        Y = torch.empty(B, 256, 256, 3, dtype=rt.dtype, device=dev)
        if out_u8 is not None and (out_u8.shape != (B, 256, 256, 3) or out_u8.dtype != torch.uint8
                                   or not out_u8.is_contiguous() or out_u8.device != dev):
            raise RuntimeError("ghost_amd: out_u8 must be a contiguous uint8 [B,256,256,3] tensor on the input device")
        lib = rt.lib
        stream = _lib.stream_ptr(dev)
        ws = rt.workspace("forward", B, dev, stream)
        ap = (C.c_void_p * 8)(*[a.data_ptr() for a in attrs])
        blocks = []
        if taps:
            cin_cout = [(1024, 1024), (1024, 1024), (1024, 1024), (1024, 512), (512, 256), (256, 128), (128, 64)]
            blocks = [torch.empty(B, 2 ** k, 2 ** k, cin_cout[k - 1][1], dtype=rt.dtype, device=dev) for k in range(1, 8)]
            _lib.check(lib.ghost_aei_set_taps(rt.h, (C.c_void_p * 8)(*[b.data_ptr() for b in blocks], None)), "taps")
        try:
            _lib.check(lib.ghost_aei_forward(rt.h, Xt.data_ptr(), _lib.gdtype(Xt.dtype), st, B, z.data_ptr(),
                                             _lib.gdtype(z.dtype), z.stride(0), Y.data_ptr(),
                                             out_u8.data_ptr() if out_u8 is not None else None, ap, ws.data_ptr(),
                                             ws.numel(), stream), "AEI_Net.forward")
        finally:
            if taps:
                lib.ghost_aei_set_taps(rt.h, None)
        od = self._out_dtype(rt)
        Y = Y.permute(0, 3, 1, 2)
        attrs = tuple(a.permute(0, 3, 1, 2) for a in attrs)
        if od != rt.dtype:
            Y, attrs = Y.to(od), tuple(a.to(od) for a in attrs)
        return Y, attrs, [b.permute(0, 3, 1, 2) for b in blocks]

    @torch.no_grad()
    def get_attr(self, X):
        rt, B, attrs, st = self._prep(X, "AEI_Net.get_attr")
        lib = rt.lib
        stream = _lib.stream_ptr(X.device)
        ws = rt.workspace("forward", B, X.device, stream)
        ap = (C.c_void_p * 8)(*[a.data_ptr() for a in attrs])
        _lib.check(lib.ghost_aei_get_attr(rt.h, X.data_ptr(), _lib.gdtype(X.dtype), st, B, ap, ws.data_ptr(),
                                          ws.numel(), stream), "AEI_Net.get_attr")
        od = self._out_dtype(rt)
        return tuple(a.permute(0, 3, 1, 2).to(od) for a in attrs)

    @torch.no_grad()
    def swap_u8(self, crops_u8: torch.Tensor, z_id: torch.Tensor, out: Optional[torch.Tensor] = None):
        """Fused faceshifter_batch on device uint8 BGR crops [B,256,256,3] -> uint8 BGR [B,256,256,3]."""
        _lib.require_gpu(crops_u8, "AEI_Net.swap_u8")
        if crops_u8.dtype != torch.uint8 or crops_u8.ndim != 4 or tuple(crops_u8.shape[1:]) != (256, 256, 3):
            raise RuntimeError("ghost_amd: crops must be uint8 [B,256,256,3]")
        if crops_u8[0].stride() != (768, 3, 1):
            crops_u8 = crops_u8.contiguous()
        dev = crops_u8.device
        _lib.require_same_device(z_id, dev, "z_id")
        rt = self._runtime(dev)
        B = crops_u8.shape[0]
        z = z_id.reshape(z_id.shape[0], -1)
        if z.stride(1) != 1:
            z = z.contiguous()
        zrs = z.stride(0) if z.shape[0] == B else 0   # one identity row broadcast (faceshifter_run.py:15-16)
        if z.shape[0] not in (1, B):
            raise RuntimeError("ghost_amd: z_id must have 1 or B rows")
        if z.shape[1] != self.c_id:
            raise RuntimeError(f"ghost_amd: z_id rows must hold {self.c_id} values, got {tuple(z_id.shape)}")
        if out is None:
            out = torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev)
        elif (tuple(out.shape) != (B, 256, 256, 3) or out.dtype != torch.uint8 or not out.is_contiguous()
              or out.device != dev):
            raise RuntimeError(f"ghost_amd: out must be a contiguous uint8 [{B},256,256,3] tensor on {dev}, got "
                               f"{out.dtype} {tuple(out.shape)} on {out.device}")
        lib = rt.lib
        stream = _lib.stream_ptr(dev)
        ws = rt.workspace("swap", B, dev, stream)
        cstride = crops_u8.stride(0) if B > 1 else 256 * 256 * 3     # a single crop: any dim-0 stride (a[None])
        _lib.check(lib.ghost_aei_swap_u8(rt.h, crops_u8.data_ptr(), cstride, B, z.data_ptr(),
                                         _lib.gdtype(z.dtype), zrs, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                         stream), "AEI_Net.swap_u8")
        return out

    @torch.no_grad()
    def identity_table(self, source_embeds: torch.Tensor) -> "IdentityTable":
        """The per-identity projection table of ``source_embeds`` ([n, c_id] rows on the device, any float dtype):
        every AADLayer's fc1/fc2 (gamma_id, beta_id; AADLayer.py:28-29) and up1 (AEI_Net.py:101) of each source
        embedding, computed once (``ghost_aei_identity_table``) for the module's current weights.  A video's source
        identity is the same for every frame (faceshifter_run.py:15-16 repeats one z_id over the batch), so
        ``swap_u8_indexed`` then gathers each sample's rows instead of projecting the embedding per frame."""
        _lib.require_gpu(source_embeds, "AEI_Net.identity_table")
        dev = source_embeds.device
        rt = self._runtime(dev)
        z = source_embeds.reshape(source_embeds.shape[0], -1)
        if z.shape[0] < 1 or z.shape[1] != self.c_id:
            raise RuntimeError(f"ghost_amd: source_embeds must hold n >= 1 rows of {self.c_id}, got "
                               f"{tuple(source_embeds.shape)}")
        if z.stride(1) != 1:
            z = z.contiguous()
        n = z.shape[0]
        lib = rt.lib
        nb = lib.ghost_aei_identity_table_bytes(rt.h, n)
        if nb < 0:
            _lib.check(int(nb), "identity table sizing")
        buf = torch.empty(int(nb) + 256, dtype=torch.uint8, device=dev)
        off = (-buf.data_ptr()) % 256
        stream = _lib.stream_ptr(dev)
        ws = rt.workspace("idtable", n, dev, stream)
        _lib.check(lib.ghost_aei_identity_table(rt.h, z.data_ptr(), _lib.gdtype(z.dtype), z.stride(0), n,
                                                buf.data_ptr() + off, int(nb), ws.data_ptr(), ws.numel(), stream),
                   "AEI_Net.identity_table")
        return IdentityTable(rt, buf, off, n, dev)

    @torch.no_grad()
    def swap_u8_indexed(self, crops_u8: torch.Tensor, table: "IdentityTable", identity_index: torch.Tensor,
                        out: Optional[torch.Tensor] = None):
        """``swap_u8`` for a batch whose sample b swaps in identity ``identity_index[b]`` of ``table`` (config 5's
        mixed-identity batches, or one identity with an all-zero index): the identity rows are gathered from the
        table (one launch) instead of projected from per-sample z rows.  The bytes equal ``swap_u8(crops,
        source_embeds[identity_index])`` for batches of up to 64 frames (the projections are the same GEMM rows).
        ``identity_index``: int32/int64 [B]; a host tensor is range-checked here (IndexError as
        ``source_embeds[identity_index]`` would raise), a device tensor is the caller's to keep in range (an
        out-of-range value is clamped on the device, never read out of bounds)."""
        _lib.require_gpu(crops_u8, "AEI_Net.swap_u8_indexed")
        if crops_u8.dtype != torch.uint8 or crops_u8.ndim != 4 or tuple(crops_u8.shape[1:]) != (256, 256, 3):
            raise RuntimeError("ghost_amd: crops must be uint8 [B,256,256,3]")
        if crops_u8[0].stride() != (768, 3, 1):
            crops_u8 = crops_u8.contiguous()
        dev = crops_u8.device
        if not isinstance(table, IdentityTable):
            raise TypeError("ghost_amd: table must come from AEI_Net.identity_table")
        rt = self._runtime(dev)
        if table.rt is not rt or table.device != dev:
            raise RuntimeError("ghost_amd: the identity table was built for other weights or another device (the "
                               "module was re-packed since: load_state_dict / .to / .half / a parameter change); "
                               "rebuild it with identity_table")
        B = crops_u8.shape[0]
        idx = identity_index.reshape(-1)
        if idx.shape[0] != B:
            raise RuntimeError(f"ghost_amd: identity_index must hold {B} entries, got {tuple(identity_index.shape)}")
        if idx.dtype not in (torch.int32, torch.int64, torch.int16, torch.uint8):
            raise TypeError(f"ghost_amd: identity_index must be an integer tensor, got {idx.dtype}")
        if idx.device.type == "cpu":
            if B and (int(idx.min()) < 0 or int(idx.max()) >= table.n):
                raise IndexError(f"ghost_amd: identity_index out of range for {table.n} identities")
            idx = idx.to(torch.int32).to(dev)
        else:
            _lib.require_same_device(idx, dev, "identity_index")
            if idx.dtype != torch.int32 or not idx.is_contiguous():
                idx = idx.to(torch.int32).contiguous()
        if out is None:
            out = torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev)
        elif (tuple(out.shape) != (B, 256, 256, 3) or out.dtype != torch.uint8 or not out.is_contiguous()
              or out.device != dev):
            raise RuntimeError(f"ghost_amd: out must be a contiguous uint8 [{B},256,256,3] tensor on {dev}, got "
                               f"{out.dtype} {tuple(out.shape)} on {out.device}")
        lib = rt.lib
        stream = _lib.stream_ptr(dev)
        ws = rt.workspace("swap", B, dev, stream)
        cstride = crops_u8.stride(0) if B > 1 else 256 * 256 * 3
        _lib.check(lib.ghost_aei_swap_u8_indexed(rt.h, crops_u8.data_ptr(), cstride, B, table.ptr, table.n,
                                                 table.nbytes, idx.data_ptr(), out.data_ptr(), ws.data_ptr(),
                                                 ws.numel(), stream),
                   "AEI_Net.swap_u8_indexed")
        return out

    def profile(self, class_mask: int):
        """Enable per-kernel-class HIP-event timing on the native runtime (bench instrumentation)."""
        rt = self._rt
        if rt is None:
            raise RuntimeError("ghost_amd: run one forward before enabling profiling")
        _lib.check(rt.lib.ghost_aei_profile(rt.h, class_mask))

    def profile_clock(self):
        """Class 1's in-kernel clock: (total microseconds of kernel execution span, launches)."""
        rt = self._rt
        us, n = C.c_double(), C.c_int64()
        _lib.check(rt.lib.ghost_aei_profile_clock(rt.h, C.byref(us), C.byref(n), None))
        return us.value, n.value

    def kernel_variant(self, what: str = "aad_dual_256") -> str:
        """Which generation of the profiled roofline AAD kernel ran last ('v4' / 'v5')."""
        rt = self._rt
        us, n, v = C.c_double(), C.c_int64(), C.c_int()
        _lib.check(rt.lib.ghost_aei_profile_clock(rt.h, C.byref(us), C.byref(n), C.byref(v)))
        return f"v{v.value}"

    def profile_read(self, cls: int):
        rt = self._rt
        ms, n, by, fl = C.c_double(), C.c_int64(), C.c_double(), C.c_double()
        _lib.check(rt.lib.ghost_aei_profile_read(rt.h, cls, C.byref(ms), C.byref(n), C.byref(by), C.byref(fl)))
        return {"ms": ms.value, "launches": n.value, "bytes": by.value, "flops": fl.value}
