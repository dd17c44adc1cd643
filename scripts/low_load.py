"""The low-load probes of engine/probe.py on Qwen2-7B (random weights), without the rest of the bench:
python scripts/low_load.py --out gpurun_out/low_load.json"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from githubrepostorag_amd.engine.probe import run_low_load  # noqa: E402
from githubrepostorag_amd.engine.tokenizer import load_tokenizer  # noqa: E402
from githubrepostorag_amd.models import build_decoder  # noqa: E402
from githubrepostorag_amd.models.configs import decoder_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="qwen2-7b")
ap.add_argument("--batches", default="1,4,16")
ap.add_argument("--ctxs", default="1024,4096,11600")
ap.add_argument("--quant", default="none", choices=["none", "w4"],
                help="w4: the reference's precision (AWQ-format W4A16 decode GEMMs, model.quantize_w4)")
ap.add_argument("--out", default=None)
a = ap.parse_args()
cfg = decoder_config(a.model)
model = build_decoder(cfg, device=torch.device("cuda", 0), seed=1)
tok = load_tokenizer(None, cfg.vocab_size)
if a.quant == "w4":
    print(f"W4A16 decode weights: {model.quantize_w4() / 1e9:.2f} GB", flush=True)
res = run_low_load(model, tok, batches=tuple(int(b) for b in a.batches.split(",")),
                   ctxs=tuple(int(c) for c in a.ctxs.split(",")), kv_cache_gb=12.0,
                   log=lambda m: print(m, flush=True))
print(json.dumps(res))
if a.out:
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
