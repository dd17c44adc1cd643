"""Prefill-GEMM throughput of the Qwen2-7B projections at chunk sizes M
(the engine's prefill chunks are <= 16384 tokens): TFLOP/s of the library
GEMM with the tuned TunableOp table (what the engine runs) and without it,
random bf16 operands, interleaved rounds in one process."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.ops.linear import enable_tuned_gemms, linear  # noqa: E402
from scripts.microbench import rounds  # noqa: E402

SHAPES = {"qkv": (4608, 3584), "o_proj": (3584, 3584), "gate_up": (37888, 3584), "down": (3584, 18944)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="4096,8192,16384")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    tuned = enable_tuned_gemms()
    out = {"tuned_table_loaded": bool(tuned)}
    for M in map(int, a.M.split(",")):
        for name in a.shapes.split(","):
            N, K = SHAPES[name]
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            b = torch.randn(N, device=dev, dtype=torch.bfloat16) * 0.02 if name == "qkv" else None
            r = rounds({"engine_linear": lambda: linear(x, w, b)}, n=3, iters=10)
            fl = 2.0 * M * N * K
            for k in r:
                r[k]["TFLOP_s"] = round(fl / (r[k]["min_us"] * 1e-6) / 1e12, 1)
            out[f"{name}_M{M}"] = r
            print(name, M, r, flush=True)
            del x, w
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
