"""Checkpoint I/O for the engine: Hugging Face Llama safetensors <-> LlamaModel.

The benchmark runs on seeded random weights (no checkpoints offline), but a user switching from
the reference needs real models, so the engine loads the standard Hugging Face Llama layout:

    model.embed_tokens.weight, model.norm.weight, lm_head.weight (or tied to the embedding),
    model.layers.{i}.input_layernorm.weight, .post_attention_layernorm.weight,
    model.layers.{i}.self_attn.{q,k,v,o}_proj.weight, .mlp.{gate,up,down}_proj.weight

HF checkpoints already use the rotate-half RoPE pairing our kernels implement.  Tensors are read
with ``safetensors`` (no pickle), sliced for this rank's tensor-parallel shard, fused into the
engine layouts (QKV rows, [8 gate | 8 up] blocks), the RMSNorm gains folded into the projections
that consume the normed rows (fold_gain; engine/model.py) and optionally quantised to fp8.
``save_hf`` writes the inverse (used by tests and to export random-init models).
"""

from __future__ import annotations

import glob
import json
import os
from typing import Dict

import torch

from ..ops.reference import Fp8Weight, interleave_gate_up, split_gate_up


def _open_shards(path: str):
    from safetensors import safe_open
    files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
    if not files:
        raise FileNotFoundError("no *.safetensors under %s" % path)
    index: Dict[str, str] = {}
    handles = {}
    for f in files:
        h = safe_open(f, framework="pt", device="cpu")
        handles[f] = h
        for k in h.keys():
            index[k] = f
    return index, handles


def load_hf(model, path: str) -> None:
    """Fill ``model`` (an engine.model.LlamaModel) from a HF Llama safetensors checkpoint."""
    index, handles = _open_shards(path)
    cfg, dev, dt = model.cfg, model.device, model.dtype
    r = model.tp_rank

    def get(name: str) -> torch.Tensor:
        if name not in index:
            raise KeyError("checkpoint %s has no tensor %s" % (path, name))
        return handles[index[name]].get_tensor(name)

    def put(t: torch.Tensor) -> torch.Tensor:
        return t.to(device=dev, dtype=dt).contiguous()

    hd = cfg.head_dim
    qs, ks = model.hq * hd, model.hkv * hd
    f = model.ffn_local
    model.embed = put(get("model.embed_tokens.weight"))
    lm = get("lm_head.weight") if "lm_head.weight" in index else get("model.embed_tokens.weight")
    v = model.vocab_local
    model.final_norm = put(get("model.norm.weight"))
    model.lm_head = put(fold_gain(lm[r * v:(r + 1) * v], model.final_norm))
    model._quantize_lm_head()
    for i, lw in enumerate(model.layers):
        p = "model.layers.%d." % i
        lw.ln1 = put(get(p + "input_layernorm.weight"))
        lw.ln2 = put(get(p + "post_attention_layernorm.weight"))
        wq, wk, wv = (get(p + "self_attn.%s_proj.weight" % n) for n in ("q", "k", "v"))
        wqkv = torch.cat([wq[r * qs:(r + 1) * qs], wk[r * ks:(r + 1) * ks], wv[r * ks:(r + 1) * ks]])
        wo = get(p + "self_attn.o_proj.weight")[:, r * qs:(r + 1) * qs]
        wg, wu = get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight")
        wgu = interleave_gate_up(wg[r * f:(r + 1) * f], wu[r * f:(r + 1) * f])
        wd = get(p + "mlp.down_proj.weight")[:, r * f:(r + 1) * f]
        # norm gains folded into the consumer projections (engine/model.py), before fp8 quantisation
        mats = [put(t) for t in (fold_gain(wqkv, lw.ln1), wo, fold_gain(wgu, lw.ln2), wd)]
        if model.weight_dtype == "fp8":
            mats = [Fp8Weight.quantize(t) for t in mats]
        lw.wqkv, lw.wo, lw.wgu, lw.wdown = mats


def fold_gain(w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """W diag(g) in fp32, one rounding to the weight dtype (identity for an all-ones gain)."""
    g = g.to(w.device)
    if bool((g == 1).all()):
        return w
    return (w.float() * g.float()).to(w.dtype)


def unfold_gain(w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """Inverse of fold_gain for export (exact for unit gains, else within one bf16 rounding)."""
    g = g.to(w.device)
    if bool((g == 1).all()):
        return w
    return (w.float() / g.float()).to(w.dtype)


def _dense(t) -> torch.Tensor:
    return t.dequant(torch.bfloat16) if isinstance(t, Fp8Weight) else t


def save_hf(model, path: str) -> None:
    """Write a tp_size == 1 LlamaModel as a HF-layout safetensors checkpoint + config.json."""
    from safetensors.torch import save_file
    if model.tp_size != 1:
        raise ValueError("save_hf needs an unsharded model")
    cfg = model.cfg
    hd = cfg.head_dim
    qs, ks = cfg.n_heads * hd, cfg.n_kv_heads * hd
    out: Dict[str, torch.Tensor] = {
        "model.embed_tokens.weight": model.embed,
        "model.norm.weight": model.final_norm,
        "lm_head.weight": unfold_gain(_dense(model.lm_head), model.final_norm),
    }
    for i, lw in enumerate(model.layers):
        p = "model.layers.%d." % i
        wqkv = unfold_gain(_dense(lw.wqkv), lw.ln1)
        out[p + "self_attn.q_proj.weight"] = wqkv[:qs]
        out[p + "self_attn.k_proj.weight"] = wqkv[qs:qs + ks]
        out[p + "self_attn.v_proj.weight"] = wqkv[qs + ks:]
        out[p + "self_attn.o_proj.weight"] = _dense(lw.wo)
        g, u = split_gate_up(unfold_gain(_dense(lw.wgu), lw.ln2).t())
        out[p + "mlp.gate_proj.weight"] = g.t()
        out[p + "mlp.up_proj.weight"] = u.t()
        out[p + "mlp.down_proj.weight"] = _dense(lw.wdown)
        out[p + "input_layernorm.weight"] = lw.ln1
        out[p + "post_attention_layernorm.weight"] = lw.ln2
    os.makedirs(path, exist_ok=True)
    save_file({k: v.detach().to("cpu").contiguous() for k, v in out.items()}, os.path.join(path, "model.safetensors"))
    with open(os.path.join(path, "config.json"), "w") as fh:
        json.dump({"architectures": ["LlamaForCausalLM"], "hidden_size": cfg.hidden,
                   "intermediate_size": cfg.ffn, "num_hidden_layers": cfg.n_layers,
                   "num_attention_heads": cfg.n_heads, "num_key_value_heads": cfg.n_kv_heads,
                   "head_dim": cfg.head_dim, "rope_theta": cfg.rope_theta, "rms_norm_eps": cfg.rms_eps,
                   "vocab_size": cfg.vocab_size, "max_position_embeddings": cfg.max_position,
                   "torch_dtype": "bfloat16",
                   **({"rope_scaling": {"rope_type": "llama3", "factor": cfg.rope_scaling[0],
                                        "low_freq_factor": cfg.rope_scaling[1],
                                        "high_freq_factor": cfg.rope_scaling[2],
                                        "original_max_position_embeddings": cfg.rope_scaling[3]}}
                      if cfg.rope_scaling else {})}, fh, indent=1)


def config_from_hf(path: str, name: str = "hf"):
    """ModelConfig from a HF config.json (directory or file)."""
    from .config import ModelConfig
    f = os.path.join(path, "config.json") if os.path.isdir(path) else path
    with open(f) as fh:
        c = json.load(fh)
    heads = c["num_attention_heads"]
    rs = c.get("rope_scaling") or None
    scaling = None
    if rs:
        kind = rs.get("rope_type", rs.get("type"))
        if kind != "llama3":
            raise ValueError("unsupported rope_scaling %r (only Llama-3.1 'llama3' scaling)" % kind)
        scaling = (float(rs["factor"]), float(rs.get("low_freq_factor", 1.0)), float(rs.get("high_freq_factor", 4.0)),
                   int(rs.get("original_max_position_embeddings", 8192)))
    return ModelConfig(name, rope_scaling=scaling, vocab_size=c["vocab_size"], hidden=c["hidden_size"], n_layers=c["num_hidden_layers"],
                       n_heads=heads, n_kv_heads=c.get("num_key_value_heads", heads),
                       head_dim=c.get("head_dim", c["hidden_size"] // heads), ffn=c["intermediate_size"],
                       rope_theta=float(c.get("rope_theta", 500000.0)), rms_eps=float(c.get("rms_norm_eps", 1e-5)),
                       max_position=int(c.get("max_position_embeddings", 8192)))
