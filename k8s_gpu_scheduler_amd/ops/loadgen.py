"""Torch-facing wrappers for the HIP load kernels (native/hip/loadgen.hip).

`gemm(a, bt)` computes act(a @ bt.T + bias) in bf16 on MFMA, `gemm_fp8` the same with OCP
e4m3fn operands on the block-scaled fp8 MFMA; `triad(a, b, c, s)` streams HBM.  Shapes are validated on the host before launch (the kernels have no bounds checks
by design).  On a GPU box the native module is mandatory: there is no PyTorch fallback
path here (tests compare against torch fp32 references instead).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native

BM, BN, BK = 64, 64, 64          # minimum granularity; the tile (128x128 / 64x128 / 64x64) is picked per shape


def _stream_ptr(stream: Optional[torch.cuda.Stream], device: Optional[torch.device] = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    if device is not None and s.device != device:
        raise ValueError(f"stream is on {s.device}, operands on {device}")
    return int(s.cuda_stream)


def _check_devices(name: str, *ts: Optional[torch.Tensor]) -> torch.device:
    """Every operand (and output/bias when given) must be a device tensor on ONE GPU: a host
    pointer handed to the kernel is a GPU memory fault (XNACK off), another GPU's pointer
    a launch on the wrong device."""
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError(f"{name} expects device tensors (got a {t.device} tensor)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"{name}: operands on different devices ({dev} vs {t.device})")
    return dev


def check_gemm_shapes(M: int, N: int, K: int) -> None:
    if M <= 0 or N <= 0 or K <= 0 or M % BM or N % BN or K % BK:
        raise ValueError(f"gemm shape ({M},{N},{K}) must be positive multiples of ({BM},{BN},{BK})")


def gemm(a: torch.Tensor, bt: torch.Tensor, out: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
         relu: bool = False, stream: Optional[torch.cuda.Stream] = None, cu_budget: int = 0) -> torch.Tensor:
    """out[M,N] = act(a[M,K] @ bt[N,K]^T + bias[N]) -- bf16 in/out, fp32 accumulate.
    cu_budget: CUs this GEMM can expect to own (the pod's share when pods co-run; 0 = the
    whole chip) -- steers the tile choice (native pick_gemm_tile)."""
    if a.dtype != torch.bfloat16 or bt.dtype != torch.bfloat16:
        raise TypeError("gemm expects bf16 operands")
    _check_devices("gemm", a, bt, out, bias)
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ValueError(f"gemm shape mismatch {tuple(a.shape)} x {tuple(bt.shape)}^T")
    if a.stride(1) != 1 or bt.stride(1) != 1:
        raise ValueError("gemm expects row-major (K-contiguous) operands")
    M, K = a.shape
    N = bt.shape[0]
    check_gemm_shapes(M, N, K)
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if out.shape != (M, N) or out.dtype != torch.bfloat16 or out.stride(1) != 1:
        raise ValueError("bad output tensor")
    bptr = 0
    if bias is not None:
        if bias.dtype != torch.float32 or bias.numel() != N or not bias.is_contiguous():
            raise ValueError("bias must be a contiguous fp32 vector of length N")
        bptr = bias.data_ptr()
    h = _native.hip()
    with torch.cuda.device(a.device):
        sp = _stream_ptr(stream, a.device)
        # split-K (lone GEMMs whose 256x256 tiles leave CUs idle): an fp32 partial workspace from
        # the caching allocator, allocated on the launch stream so its reuse is ordered after
        # the reduce kernel
        wsf = h.splitk_workspace_floats(M, N, K, cu_budget)
        ws = None
        if wsf:
            with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream(a.device)):
                ws = torch.empty(wsf, dtype=torch.float32, device=a.device)
        h.gemm_bf16_nt(a.data_ptr(), bt.data_ptr(), out.data_ptr(), bptr, M, N, K, a.stride(0), bt.stride(0),
                       out.stride(0), relu, sp, cu_budget, ws.data_ptr() if ws is not None else 0, wsf)
    return out


FP8 = torch.float8_e4m3fn          # OCP e4m3 (gfx950), not the MI300 "fnuz" encoding


def gemm_fp8(a: torch.Tensor, bt: torch.Tensor, out: Optional[torch.Tensor] = None,
             bias: Optional[torch.Tensor] = None, relu: bool = False, stream: Optional[torch.cuda.Stream] = None,
             cu_budget: int = 0) -> torch.Tensor:
    """out[M,N] = act(a[M,K] @ bt[N,K]^T + bias[N]) -- e4m3fn operands, fp32 accumulate, bf16
    out, on the block-scaled fp8 MFMA (unit scales).  M, N multiples of 64, K of 128."""
    if a.dtype != FP8 or bt.dtype != FP8:
        raise TypeError("gemm_fp8 expects float8_e4m3fn operands")
    _check_devices("gemm_fp8", a, bt, out, bias)
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ValueError(f"gemm_fp8 shape mismatch {tuple(a.shape)} x {tuple(bt.shape)}^T")
    if a.stride(1) != 1 or bt.stride(1) != 1 or a.stride(0) % 16 or bt.stride(0) % 16:
        raise ValueError("gemm_fp8 expects row-major operands with 16-byte aligned rows")
    M, K = a.shape
    N = bt.shape[0]
    if M <= 0 or N <= 0 or K <= 0 or M % 64 or N % 64 or K % 128:
        raise ValueError(f"gemm_fp8 shape ({M},{N},{K}) must be positive multiples of (64,64,128)")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if out.shape != (M, N) or out.dtype != torch.bfloat16 or out.stride(1) != 1:
        raise ValueError("bad output tensor")
    bptr = 0
    if bias is not None:
        if bias.dtype != torch.float32 or bias.numel() != N or not bias.is_contiguous():
            raise ValueError("bias must be a contiguous fp32 vector of length N")
        bptr = bias.data_ptr()
    with torch.cuda.device(a.device):
        _native.hip().gemm_fp8_nt(a.data_ptr(), bt.data_ptr(), out.data_ptr(), bptr, M, N, K, a.stride(0),
                                  bt.stride(0), out.stride(0), relu, _stream_ptr(stream, a.device), cu_budget)
    return out


def triad(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, s: float = 1.5, blocks: int = 0,
          stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """a = b + s*c (fp32, contiguous, numel % 4 == 0)."""
    _check_devices("triad", a, b, c)
    for t in (a, b, c):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("triad expects contiguous fp32 device tensors")
    n = a.numel()
    if b.numel() != n or c.numel() != n or n % 4:
        raise ValueError("triad: sizes must match and be a multiple of 4")
    with torch.cuda.device(a.device):
        _native.hip().stream_triad(a.data_ptr(), b.data_ptr(), c.data_ptr(), float(s), n, int(blocks),
                                   _stream_ptr(stream, a.device))
    return a


def gemm_flops(M: int, N: int, K: int) -> float:
    return 2.0 * M * N * K
