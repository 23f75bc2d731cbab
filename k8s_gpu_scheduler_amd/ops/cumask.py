"""CU-masked HIP streams (fractional GPU sharing) and the XCD map probe.

A fractional pod granted CU-slice units [u0, u0+n) of a device (unit u = word u of the
256-bit CU mask = 4 CUs on each of the 8 XCDs) runs its kernels on a `MaskedStream`
whose hardware queue only dispatches to those CUs (hipExtStreamCreateWithCUMask,
native/hip/cumask.hip).  `probe_xcd_map` launches a probe kernel under a mask and
reports which XCC ids / CUs executed it -- how the bit -> (XCC, CU) mapping assumed by
`plugins.gpu.devices.cu_slice_mask` was established on MI355X (bit i -> XCC i % 8; a mask
leaving an XCC empty is ignored by the driver).
"""
from __future__ import annotations

from collections import Counter
from typing import Dict, List, Optional, Sequence

import torch

from .. import _native
from ..plugins.gpu.devices import cu_slice_mask


class MaskedStream:
    def __init__(self, mask_words: Sequence[int], device: Optional[int] = None):
        self.mask = [int(w) & 0xFFFFFFFF for w in mask_words]
        dev = torch.cuda.current_device() if device is None else device
        with torch.cuda.device(dev):
            self.ptr = _native.hip().create_masked_stream(self.mask)
            self.stream = torch.cuda.ExternalStream(self.ptr, device=torch.device("cuda", dev))
        self.device = dev

    @classmethod
    def for_units(cls, first_unit: int, n_units: int, device: Optional[int] = None) -> "MaskedStream":
        return cls(cu_slice_mask(first_unit, n_units), device)

    def close(self) -> None:
        if self.ptr:
            torch.cuda.synchronize(self.device)
            _native.hip().destroy_stream(self.ptr)
            self.ptr = 0

    def __del__(self) -> None:  # best effort
        try:
            if self.ptr and torch.cuda.is_available():
                _native.hip().destroy_stream(self.ptr)
                self.ptr = 0
        except Exception:
            pass


def probe_xcd_map(mask_words: Optional[Sequence[int]] = None, blocks: int = 4096) -> Dict[str, object]:
    """Run the probe kernel (optionally under a mask); returns the XCC ids hit and the
    number of distinct (xcc, se, cu) slots per XCC."""
    h = _native.hip()
    if mask_words is None:
        s = torch.cuda.current_stream()
        raw = h.probe_xcd(int(s.cuda_stream), blocks)
    else:
        ms = MaskedStream(mask_words)
        try:
            raw = h.probe_xcd(ms.ptr, blocks)
        finally:
            ms.close()
    xcc = [raw[2 * i] & 0xF for i in range(blocks)]
    hw = [raw[2 * i + 1] for i in range(blocks)]
    cus_per_xcc: Dict[int, set] = {}
    for x, w in zip(xcc, hw):
        cu = (w >> 8) & 0xF
        sh = (w >> 12) & 0x1
        se = (w >> 13) & 0x7
        cus_per_xcc.setdefault(x, set()).add((se, sh, cu))
    return {"xcc_hist": dict(sorted(Counter(xcc).items())),
            "cus_per_xcc": {k: len(v) for k, v in sorted(cus_per_xcc.items())}}


def verify_unit_masks(units_per_slot: int = 2) -> List[Dict[str, object]]:
    """For each aligned slot of `units_per_slot` mask words, probe which XCCs/CUs execute
    (expected: all 8 XCCs, 4*units_per_slot CUs each)."""
    out = []
    for first in range(0, 8, units_per_slot):
        r = probe_xcd_map(cu_slice_mask(first, units_per_slot))
        r["slot_units"] = list(range(first, first + units_per_slot))
        out.append(r)
    return out
