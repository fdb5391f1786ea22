"""Device placement of compiled weights, and weight sharing between replicas.

Every fused op moves its (folded) weights to the device through
:func:`to_device`.  A replica that receives its weights over RCCL
(``parallel/weights.py``) compiles the program from a *meta* bundle -- tensors
with shapes and dtypes but no data -- so folding runs on shapes only and
:func:`to_device` turns each meta weight into an uninitialised device tensor
(no host->device copy).  :func:`weight_refs` then finds every weight tensor
the compiled program holds, in a deterministic order that is identical on
every replica compiling the same graph with the same passes;
:func:`export_weights` packs them into ONE contiguous device blob (the RCCL
broadcast unit) and :func:`bind_weights` re-points a program's
tensors at views of a received blob.

``H2D_BYTES`` counts the weight bytes actually copied host -> device by
:func:`to_device` (tests assert a follower's load adds none).
"""
from __future__ import annotations

import threading
from typing import List, Optional, Tuple

import torch

_LOCK = threading.Lock()
H2D_BYTES = 0


def to_device(t: torch.Tensor, device, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """``t.to(device, dtype).contiguous()``; a meta tensor becomes an empty
    device tensor of its shape (filled later by :func:`bind_weights`)."""
    global H2D_BYTES
    dev = torch.device(device) if device is not None else t.device
    want = dtype or t.dtype
    if t.is_meta:
        if dev.type == "meta":
            return t.to(want)
        return torch.empty(t.shape, dtype=want, device=dev)
    if t.device != dev and dev.type != "cpu" and t.device.type == "cpu":
        with _LOCK:
            H2D_BYTES += t.numel() * torch.empty((), dtype=want).element_size()
    return t.to(device=dev, dtype=want).contiguous()


def zeros(n, like: torch.Tensor, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """``torch.zeros`` on ``like``'s device (meta stays meta)."""
    return torch.zeros(n, dtype=dtype or torch.float32, device=like.device)


# ------------------------------------------------------------------ weight refs
Ref = Tuple[object, str, Optional[int]]        # (holder, attribute / const slot, index in a tuple/list)


def _tensor_attrs(obj) -> List[Tuple[str, Optional[int], torch.Tensor]]:
    out = []
    for k in sorted(vars(obj)):
        v = getattr(obj, k)
        if isinstance(v, torch.Tensor):
            out.append((k, None, v))
        elif isinstance(v, (tuple, list)):
            for i, x in enumerate(v):
                if isinstance(x, torch.Tensor):
                    out.append((k, i, x))
    return out


def weight_refs(program) -> List[Tuple[Ref, torch.Tensor]]:
    """Every weight-like tensor the program holds on its device: tensors in
    the fused-op implementations (in step order, attributes sorted) and the
    device-resident constant slots."""
    dev = program.device
    out = []
    seen = set()

    def visit(impl):
        if impl is None or id(impl) in seen:
            return
        seen.add(id(impl))
        for k, i, t in _tensor_attrs(impl):
            if (t.device.type == dev.type or t.is_meta) and t.numel() > 0:
                out.append(((impl, k, i), t))
        for child in getattr(impl, "children", ()):   # fused ops built from other fused ops
            visit(getattr(impl, child))

    for fn, node, _ins, _outs in program.steps:
        visit(node.attrs.get("_impl"))
    for pos, (slot, v) in enumerate(program.const_slots):
        # a follower's host program keeps shape-only (meta) weights until bound
        if isinstance(v, torch.Tensor) and (v.device.type == dev.type or v.is_meta) and v.numel() > 0 and \
                (v.is_floating_point() or v.is_meta or dev.type != "cpu"):
            out.append(((program, "const_slots", pos), v))
    return out


def _set(ref: Ref, value: torch.Tensor) -> None:
    holder, k, i = ref
    if k == "const_slots":
        slot, _old = holder.const_slots[i]
        holder.const_slots[i] = (slot, value)
        return
    if i is None:
        setattr(holder, k, value)
        return
    seq = getattr(holder, k)
    lst = list(seq)
    lst[i] = value
    setattr(holder, k, tuple(lst) if isinstance(seq, tuple) else lst)


def manifest_of(refs) -> List[Tuple[str, Tuple[int, ...], int, int]]:
    """[(dtype name, shape, byte offset, nbytes)], 256-B aligned offsets."""
    man, off = [], 0
    for _ref, t in refs:
        nb = t.numel() * t.element_size()
        man.append((str(t.dtype).replace("torch.", ""), tuple(t.shape), off, nb))
        off += (nb + 255) // 256 * 256
    return man


def blob_bytes(manifest) -> int:
    return max(1, max((o + n for _d, _s, o, n in manifest), default=0))


def export_weights(program) -> Tuple[torch.Tensor, list]:
    """Pack the program's weights into one device blob (device-to-device
    copies) and re-point the program at views of it; returns (blob, manifest)."""
    refs = weight_refs(program)
    man = manifest_of(refs)
    blob = torch.empty(blob_bytes(man), dtype=torch.uint8, device=program.device)
    for (ref, t), (_d, _s, off, nb) in zip(refs, man):
        view = blob[off:off + nb].view(t.dtype).view(t.shape)
        view.copy_(t)
        _set(ref, view)
    return blob, man


def bind_weights(program, blob: torch.Tensor, manifest) -> int:
    """Re-point ``program``'s weights at views of ``blob`` (a replica of the
    leader's program); returns the bytes bound.  Shapes / dtypes must match."""
    refs = weight_refs(program)
    if len(refs) != len(manifest):
        raise ValueError(f"weight manifest has {len(manifest)} tensors, the program {len(refs)}")
    total = 0
    for (ref, t), (dname, shape, off, nb) in zip(refs, manifest):
        dt = getattr(torch, dname)
        if tuple(t.shape) != tuple(shape) or t.dtype != dt:
            raise ValueError(f"weight mismatch: program {tuple(t.shape)} {t.dtype} vs manifest {shape} {dname}")
        _set(ref, blob[off:off + nb].view(dt).view(shape))
        total += nb
    return total
