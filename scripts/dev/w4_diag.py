"""Root-cause probe for the W4A16 kernel's 4/8/12-row-tile variants (VERDICT r2 missing 6).

Builds (``--build``, on the CPU host) diagnostic copies of csrc/kernels/gemm_w4.hip with every row
tiling enabled and one behaviour changed per copy (GRAG_W4_DIAG bits, see the kernel source):
  d0  as shipped                               (loads in flight across the barrier, LDS sized to the ring)
  d1  every load drained before the barrier    (no in-flight register / LDS-DMA writes during compute)
  d2  LDS padded to 160 KB                     (one workgroup per CU)
  d4  weights by plain compiler-visible loads (no inline-asm register ring; hipcc places the waits)
  d5  d4 + drain before the barrier
  d8  in-kernel checks: every A fragment read from the LDS ring and every W word from the register ring
      compared with the same bytes loaded straight from global memory (mismatch counters + first
      mismatch's step / tile / lane), d12 the same with plain W loads
  d16 16 wait states between the dequant (VALU writes of the W fragments) and the MFMAs reading them,
      d17 the same + drain before the barrier
and (``--run``, on the GPU) times nothing: it runs each copy on dense random operands for every tiling
and reports the max relative error against the fp32 reference of the same 4-bit weights, several times
in one process.  Which switch removes the error names the mechanism.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "scripts", "dev", "_w4diag")  # the .so files travel to the GPU box (build/ does not)
OBJ = os.path.join(ROOT, "build", "w4diag")
sys.path.insert(0, ROOT)
DIAGS = (0, 1, 16, 17)


def build():
    from githubrepostorag_amd.utils.native_build import HIPCC_FLAGS, _hipcc

    os.makedirs(OUT, exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    hipcc = _hipcc()
    k = os.path.join(ROOT, "csrc", "kernels")
    tile_o = os.path.join(OBJ, "gemm_tile.o")
    subprocess.run([hipcc, *HIPCC_FLAGS, "-I", k, "-c", os.path.join(k, "gemm_tile.hip"), "-o", tile_o], check=True)
    for d in DIAGS:
        o = os.path.join(OBJ, f"w4_d{d}.o")
        subprocess.run([hipcc, *HIPCC_FLAGS, "-I", k, f"-DGRAG_W4_DIAG={d}", "-DGRAG_W4_ALL_VARIANTS", "-c",
                        os.path.join(k, "gemm_w4.hip"), "-o", o], check=True)
        subprocess.run([hipcc, HIPCC_FLAGS[0], "-shared", "-fPIC", "-o", os.path.join(OUT, f"libw4_d{d}.so"), o,
                        tile_o], check=True)
    print("built", sorted(os.listdir(OUT)))


def run(reps: int):
    import torch

    from githubrepostorag_amd.ops.w4 import W4Linear

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = [(64, 3584, 3584), (128, 4608, 3584), (192, 3584, 3584), (256, 3584, 3584)]
    P, I = ctypes.c_void_p, ctypes.c_int
    for d in DIAGS:
        lib = ctypes.CDLL(os.path.join(OUT, f"libw4_d{d}.so"), mode=ctypes.RTLD_LOCAL)
        f = lib.grag_gemm_w4
        f.argtypes = [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P]
        f.restype = I
        for M, N, K in shapes:
            w = (torch.randn(N, K, generator=g) * 0.05).to(dev)
            q = W4Linear.quantize(w)
            ref_w = q.dequant(torch.float32)
            x = (torch.randn(M, K, generator=g)).to(dev).to(torch.bfloat16)
            ref = x.float() @ ref_w.t()
            for mt in (4, 8, 12, 16):
                if 16 * mt < M:
                    continue
                errs = []
                diag = None
                for _ in range(reps):
                    if d & 8:
                        lib.grag_w4_diag(None, 1)
                    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
                    rc = f(x.data_ptr(), q.wq.data_ptr(), q.sz.data_ptr(), None, out.data_ptr(), x.stride(0),
                           out.stride(0), M, N, K, 0, 0, mt, 4, 1, None, torch.cuda.current_stream().cuda_stream)
                    torch.cuda.synchronize()
                    assert rc == 0, rc
                    e = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                    errs.append(round(e, 5))
                    if d & 8:
                        buf = (ctypes.c_uint * 16)()
                        lib.grag_w4_diag(buf, 0)
                        diag = list(buf)[:9]
                print(json.dumps({"diag": d, "M": M, "N": N, "K": K, "mt": mt, "max_rel_err": max(errs),
                                  "errs": errs, "checks": diag}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    if a.build:
        build()
    if a.run:
        run(a.reps)
