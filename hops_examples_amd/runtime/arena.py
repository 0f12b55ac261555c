"""ParamArena: every trainable parameter of a model lives in ONE flat buffer.

Layout per arena (all on the model's device):
  master  fp32 [N]   the parameters (``p.data`` are views into it)
  grad    fp32 [N]   gradients; hopsx kernels ACCUMULATE into it with atomics
  shadow  bf16 [N]   the copy the MFMA kernels read; refreshed by the fused
                     optimizer in the same pass that updates ``master``
  state_k fp32 [N]   optimizer moments, allocated lazily

Why: the optimizer is one launch over the whole model, the data-parallel
all-reduce works on contiguous grad buckets with no pack/unpack copies, the
bf16 weight cast is free (fused into the optimizer) and the step has a fixed
memory footprint, which is what makes whole-step hipGraph capture possible.
Offsets are 64-element aligned so every view is 256-B aligned (16-B vector
loads in the kernels).
"""
from __future__ import annotations

import torch

ALIGN = 64


class ParamArena:
    def __init__(self, params, device=None, shadow: bool | None = None, pad_multiple: int = ALIGN):
        params = [p for p in params if p.requires_grad]
        seen, uniq = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params = uniq
        if device is None:
            device = uniq[0].device if uniq else torch.device("cpu")
        self.device = torch.device(device)
        offs, n = [], 0
        for p in uniq:
            offs.append(n)
            n += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        pad = max(ALIGN, int(pad_multiple))
        self.numel = max(-(-n // pad) * pad, pad)  # sharded (PS) modes need numel % (world*ALIGN) == 0
        self.offsets = offs
        self.master = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        self.grad = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        if shadow is None:
            shadow = self.device.type == "cuda"
        self.shadow = torch.zeros(self.numel, device=self.device, dtype=torch.bfloat16) if shadow else None
        self.states: dict[str, torch.Tensor] = {}
        with torch.no_grad():
            for p, o in zip(uniq, offs):
                k = p.numel()
                self.master[o:o + k].copy_(p.detach().reshape(-1).to(self.device, torch.float32))
                p.data = self.master[o:o + k].view(p.shape)
                p._hx_grad = self.grad[o:o + k].view(p.shape)
                p._hx_off = o
                p._hx_arena = self
                if self.shadow is not None:
                    p._hx_shadow = self.shadow[o:o + k].view(p.shape)
                p.grad = p._hx_grad
                # params updated by plain torch ops (not hopsx kernels) get their
                # grad folded into the arena after autograd accumulates it
                if hasattr(p, "register_post_accumulate_grad_hook") and not getattr(p, "_hx_hooked", False):
                    p.register_post_accumulate_grad_hook(_fold_grad)
                    p._hx_hooked = True
        self.refresh_shadow()

    # ------------------------------------------------------------------ api
    @classmethod
    def from_module(cls, module: torch.nn.Module, device=None, pad_multiple: int = ALIGN) -> "ParamArena":
        if device is not None:
            module.to(device)
        arena = cls(list(module.parameters()), device=device, pad_multiple=pad_multiple)
        module._hx_arena = arena
        return arena

    def refresh_shadow(self) -> None:
        if self.shadow is None:
            return
        if self.device.type == "cuda":
            from ..ops import kernels as K

            K.cast_f32_bf16(self.master, out=self.shadow)
        else:
            self.shadow.copy_(self.master)

    def wire_mask(self) -> torch.Tensor | None:
        """uint8 [ceil(numel / 64)] per 64-element chunk: 1 where the chunk belongs to a parameter
        the kernels read only through the bf16 shadow (``_hx_wire_bf16``: conv / dense weights).
        The fused P2P step all-gathers those chunks in bf16 (ZeRO-1); None if there are none."""
        m = torch.zeros(-(-self.numel // ALIGN), dtype=torch.uint8)
        for p, o in zip(self.params, self.offsets):
            if getattr(p, "_hx_wire_bf16", False):
                m[o // ALIGN:-(-(o + p.numel()) // ALIGN)] = 1
        return m.to(self.device) if bool(m.any()) else None

    def rebind_grad(self, buf: torch.Tensor) -> None:
        """Move the gradient into ``buf`` (fp32, >= numel elements, same device): the zero-copy P2P step
        hands the arena memory its peers map over xGMI (parallel/oneshot.py make_grad_buffer).  Every
        parameter's ``.grad`` view is re-pointed; call before any graph capture (captured kernels keep
        the pointers they were captured with)."""
        if buf.dtype != torch.float32 or buf.numel() < self.numel or buf.device != self.device:
            raise ValueError("rebind_grad needs an fp32 buffer of >= numel elements on the arena's device")
        buf = buf[:self.numel]
        with torch.no_grad():
            buf.copy_(self.grad)
            self.grad = buf
            for p, o in zip(self.params, self.offsets):
                k = p.numel()
                p._hx_grad = self.grad[o:o + k].view(p.shape)
                p.grad = p._hx_grad

    def zero_grad(self) -> None:
        self.grad.zero_()

    def state(self, name: str) -> torch.Tensor:
        if name not in self.states:
            self.states[name] = torch.zeros(self.numel, device=self.device, dtype=torch.float32)
        return self.states[name]

    def ranges(self):
        """(param, offset, numel) in registration (= forward) order."""
        return [(p, o, p.numel()) for p, o in zip(self.params, self.offsets)]

    def state_dict(self) -> dict:
        return {"master": self.master.detach().cpu(), **{k: v.detach().cpu() for k, v in self.states.items()}}

    def load_state_dict(self, sd: dict) -> None:
        with torch.no_grad():
            self.master.copy_(sd["master"].to(self.device))
            for k, v in sd.items():
                if k != "master":
                    self.state(k).copy_(v.to(self.device))
        self.refresh_shadow()


def _fold_grad(p):
    g = p.grad
    tgt = getattr(p, "_hx_grad", None)
    if tgt is None or g is None or g.data_ptr() == tgt.data_ptr():
        return
    with torch.no_grad():
        tgt.add_(g)
    p.grad = tgt


def weight_bf16(p: torch.Tensor) -> torch.Tensor:
    """bf16 view of a parameter for the MFMA kernels (arena shadow if available)."""
    s = getattr(p, "_hx_shadow", None)
    if s is not None:
        return s
    from ..ops import kernels as K

    return K.cast_f32_bf16(p.detach().contiguous())


def grad_target(p: torch.Tensor):
    """fp32 buffer the kernels accumulate this param's gradient into, or None."""
    return getattr(p, "_hx_grad", None)
