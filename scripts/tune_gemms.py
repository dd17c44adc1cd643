"""Tune the hipBLASLt/rocBLAS solution for every plain (library) GEMM shape
the engine runs, with PyTorch TunableOp, and report default-vs-tuned times.

    python scripts/tune_gemms.py --out githubrepostorag_amd/tuning/tunableop_gfx950.csv

The engine loads the resulting CSV read-only (utils/runtime.enable_tuned_gemms),
so tuning never happens inside a timed or graph-captured region."""
import argparse
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="githubrepostorag_amd/tuning/tunableop_gfx950.csv")
ap.add_argument("--model", default="qwen2-7b")
ap.add_argument("--encoder", default="bge-large-en-v1.5")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.abspath(a.out)
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "60")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.models.configs import decoder_config, encoder_config  # noqa: E402

dc, ec = decoder_config(a.model), encoder_config(a.encoder)
H, I, D = dc.hidden_size, dc.intermediate_size, dc.head_dim
qkv = (dc.num_heads + 2 * dc.num_kv_heads) * D
dec_nk = [(qkv, H), (H, dc.num_heads * D), (2 * I, H), (H, I)]
EH, EI = ec.hidden_size, ec.intermediate_size
enc_nk = [(3 * EH, EH), (EH, EH), (EI, EH), (EH, EI)]
shapes = []
for M in (16384, 8192, 4096, 2048, 1024):
    shapes += [(M, n, k) for n, k in dec_nk]
for M in (16, 24, 32, 48, 64, 96, 128, 192, 256):
    shapes += [(M, n, k) for n, k in dec_nk] + [(M, dc.vocab_size, H)]
for M in (512, 1024, 2048, 4096, 8192):
    shapes += [(M, n, k) for n, k in enc_nk]
dev = torch.device("cuda")


def t(fn):
    fn()
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - s) / a.iters * 1e6


res = []
for M, N, K in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    torch.cuda.tunable.enable(False)
    base = t(lambda: torch.nn.functional.linear(x, w))
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.nn.functional.linear(x, w)  # tunes this shape
    torch.cuda.tunable.tuning_enable(False)
    tuned = t(lambda: torch.nn.functional.linear(x, w))
    tf = 2 * M * N * K / 1e12
    res.append((M, N, K, base, tuned))
    print(f"M={M:6d} N={N:6d} K={K:6d}  default {base:9.1f} us ({tf / base * 1e6:7.1f} TF)  "
          f"tuned {tuned:9.1f} us ({tf / tuned * 1e6:7.1f} TF)  x{base / tuned:.2f}", flush=True)
    del x, w
print("results are written at exit to", torch.cuda.tunable.get_filename())
