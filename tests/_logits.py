"""Shared helpers for logit-level checks: one unchunked prefill of a whole prefix through the model's
forward (paged KV in a private cache) and the tolerance rule the engine tests apply to it."""
import torch


def prefill_logits(model, ids, dev, last_only=False):
    """(logits [T, V] (or [V] for the last position), the KV cache the prefill wrote) of one unchunked
    prefill of ``ids``."""
    from githubrepostorag_amd.ops.attention import AttnMetadata

    T, bs = len(ids), 16
    nb = -(-T // bs)
    kv = model.allocate_kv_cache(nb + 4, bs)
    i32 = dict(dtype=torch.int32, device=dev)
    meta = AttnMetadata(q_start=torch.tensor([0, T], **i32), ctx_len=torch.tensor([T], **i32),
                        block_tables=torch.arange(nb, **i32).view(1, nb), slot_mapping=torch.arange(T, **i32),
                        max_q_len=T, num_seqs=1, num_tokens=T)
    with torch.no_grad():
        h = model.forward(torch.tensor(ids, **i32), torch.arange(T, **i32), meta, kv)
        if last_only:
            h = h[-1:]
        out = model.compute_logits(h).float().cpu()
    return (out[0] if last_only else out), kv


def greedy_within_tolerance(model, dev, prompt, generated, frac=0.02):
    """Every greedily generated token must be the recompute's best token up to bf16 noise: its logit in a
    prefill recompute of the full prefix is within ``frac`` x the logit scale of the recompute's maximum.
    Returns the worst (max logit - chosen logit) / scale over the tokens."""
    worst = 0.0
    for j, tok in enumerate(generated):
        lg, _ = prefill_logits(model, list(prompt) + list(generated[:j]), dev, last_only=True)
        scale = lg.abs().max().item()
        gap = (lg.max() - lg[tok]).item() / scale
        assert gap <= frac, (j, tok, int(lg.argmax()), gap)
        worst = max(worst, gap)
    return worst
