"""Host-side caching shared by the drop-in modules (AEI_Net, IResNet).

* ``PackedModule``: a module whose weights are packed once per (device, compute dtype) into the
  kernels' layouts.  The pack is reused until one of these invalidates it:
  - the key (device, dtype) changes;
  - ``load_state_dict`` runs;
  - ``_apply`` (``.to`` / ``.cuda`` / ``.half`` ...) runs on the module **or on any of its submodules**
    (every submodule's ``_apply`` is wrapped at construction to invalidate its owner);
  - a parameter, buffer or submodule is assigned anew anywhere in the tree (``m.weight = nn.Parameter(...)``,
    ``m.register_buffer(...)``: torch's global registration hooks, filtered to modules this tree owns);
  - a parameter or buffer is modified in place (its version counter moved: one C-level pass over the cached
    tensors' counters, ~30 us for AEI_Net's 311 tensors, not a ``state_dict()`` walk ~0.9 ms).
  Not detected: swapping a tensor's storage with ``p.data = t`` (no version bump, no hook); call
  ``invalidate_pack()`` after doing that.
* ``WorkspaceCache``: one device workspace per (mode, batch, stream), reused by later calls on the
  same stream.  Launches on one stream are ordered, so a call never overwrites scratch that an
  earlier call still reads; two streams (two batches in flight) get two workspaces.
"""
from __future__ import annotations

import operator
import types
import weakref
from typing import Callable

import torch
import torch.nn as nn
import torch.nn.modules.module as _tmod

_VERSION = operator.attrgetter("_version")
_OWNER = "_ghost_pack_owner"


def _owner_of(module):
    ref = module.__dict__.get(_OWNER)
    return ref() if ref is not None else None


def _on_register(module, name, value):
    """Global registration hook: a parameter / buffer / submodule assigned into a module of a packed tree."""
    root = _owner_of(module)
    if root is not None:
        root._invalidate()
        if isinstance(value, nn.Module):
            root._adopt(value)
    return None


def _owned_apply(self, fn, *args, **kwargs):
    """``_apply`` of a submodule of a packed tree (``.to`` / ``.half`` on the submodule itself)."""
    root = _owner_of(self)
    if root is not None:
        root._invalidate()
    return type(self)._apply(self, fn, *args, **kwargs)


_HOOKS_INSTALLED = False


def _install_hooks():
    global _HOOKS_INSTALLED
    if not _HOOKS_INSTALLED:
        _tmod.register_module_parameter_registration_hook(_on_register)
        _tmod.register_module_buffer_registration_hook(_on_register)
        _tmod.register_module_module_registration_hook(_on_register)
        _HOOKS_INSTALLED = True


class PackedModule(nn.Module):
    def _init_packed(self):
        self._rt = None
        self._rt_key = None        # (device, compute dtype) the runtime was packed for
        self._rt_tensors = ()      # the state_dict tensors it was packed from, and their version counters
        self._rt_versions = ()
        self.register_load_state_dict_post_hook(lambda module, keys: module._invalidate())
        _install_hooks()
        for m in self.modules():
            if m is not self:
                self._adopt(m)

    def _adopt(self, m: nn.Module):
        """Mark m (and its subtree) as owned by this packed module: assignments into it and ``m.to(...)`` /
        ``m.half()`` invalidate the pack."""
        ref = weakref.ref(self)
        for sub in m.modules():
            if sub is self:
                continue
            sub.__dict__[_OWNER] = ref
            if "_apply" not in sub.__dict__:
                # a bound method (deepcopy rebinds it to the copy), not a closure over this instance
                sub.__dict__["_apply"] = types.MethodType(_owned_apply, sub)

    def _invalidate(self):
        self._rt_key = None

    def invalidate_pack(self):
        """Force a re-pack on the next call (after ``p.data = t``, which nothing can observe cheaply)."""
        self._invalidate()

    def _apply(self, fn, *args, **kwargs):
        if hasattr(self, "_rt_key"):
            self._invalidate()
        return super()._apply(fn, *args, **kwargs)

    def _pack_current(self, rt=None) -> bool:
        """True when the cached pack (and, if given, exactly the runtime ``rt``) is still valid."""
        return (self._rt is not None and self._rt_key is not None and (rt is None or self._rt is rt)
                and tuple(map(_VERSION, self._rt_tensors)) == self._rt_versions)

    def _cached_runtime(self, device, dt, build: Callable[[dict], object]):
        """The runtime for (device, dt); ``build(state_dict)`` packs a new one when stale."""
        if self._rt_key == (device, dt) and self._pack_current():
            return self._rt
        sd = {k: v.detach() for k, v in self.state_dict().items()}
        for k, v in sd.items():
            if v.is_floating_point() and v.device != device:
                raise RuntimeError(f"ghost_amd: parameter {k} is on {v.device}, input on {device}")
        self._rt = None     # release the previous handle (and its workspaces) before allocating anew
        with torch.no_grad():
            self._rt = build(sd)
        self._rt_key = (device, dt)
        self._rt_tensors = tuple(self.state_dict().values())
        self._rt_versions = tuple(map(_VERSION, self._rt_tensors))
        return self._rt


class WorkspaceCache:
    """At most ``cap`` workspaces, least recently used evicted (each was allocated while its stream was
    current, so the caching allocator frees it stream-ordered)."""

    def __init__(self, cap: int = 4):
        self.cap = cap
        self.ws = {}

    def clear(self):
        self.ws = {}

    def get(self, key, nbytes_fn: Callable[[], int], dev: torch.device) -> torch.Tensor:
        ws = self.ws.pop(key, None)
        if ws is None:
            nbytes = int(nbytes_fn())
            while len(self.ws) >= self.cap:
                self.ws.pop(next(iter(self.ws)))
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self.ws[key] = ws
        return ws
