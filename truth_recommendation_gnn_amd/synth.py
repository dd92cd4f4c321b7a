"""Deterministic synthetic user<->post graphs with the schema ``build_graph.py`` saves.

``build_graph.py:476-486`` writes ``x`` ([U+P, 64] fp32, users first), and int64 COO relations
``edge_index_engage`` (user -> global post id), ``edge_index_social`` (follower -> followee).
``train_gnn.py:115-142`` turns that into the training graph: local post ids (``dst - U``), the
relation ``('user','engages','post')`` and its flip ``('post','rev_engages','user')``.
The real TSV inputs and the SentenceTransformer encoder are unavailable, so
this module reproduces only the output schema, seeded:

* graph seed 0, feature seed 1, weight seed 2, negative-sample seed 3 (numpy PCG64);
* user endpoints uniform, post endpoints Zipf-like ``p ∝ (rank+1)^-0.8`` over shuffled ranks;
* features N(0,1) then row-L2-normalised (mirrors ``build_graph.py:455-456``).

Config names follow BASELINE.json ``configs``: ``cfg1`` (toy, 3 relations as the reference),
``cfg2`` (1M users / 100k posts / 20M engages, d=64), ``cfg3`` (same, d=128), ``cfg4``
(9M users / 1M posts / 200M engages, d=128), ``cfg5`` (cfg4 + user-user and post-post
relations).  ``scaled(name, factor)`` shrinks a config for parity tests.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Optional, Tuple

import numpy as np
import torch

GRAPH_SEED, FEAT_SEED, WEIGHT_SEED, NEG_SEED = 0, 1, 2, 3

EdgeType = Tuple[str, str, str]
ENGAGES: EdgeType = ("user", "engages", "post")
REV_ENGAGES: EdgeType = ("post", "rev_engages", "user")
SOCIAL: EdgeType = ("user", "social", "user")
POST_POST: EdgeType = ("post", "related", "post")


@dataclasses.dataclass(frozen=True)
class GraphConfig:
    name: str
    num_users: int
    num_posts: int
    num_engages: int          # 0 => one engager per post (build_graph.py:390-394 shape)
    num_social: int
    num_post_post: int
    dim: int
    hidden: int
    layers: int
    zipf_s: float = 0.8


CONFIGS: Dict[str, GraphConfig] = {
    "cfg1": GraphConfig("cfg1", 256, 768, 0, 2048, 0, 64, 64, 1),
    "cfg2": GraphConfig("cfg2", 1_000_000, 100_000, 20_000_000, 0, 0, 64, 64, 2),
    "cfg3": GraphConfig("cfg3", 1_000_000, 100_000, 20_000_000, 0, 0, 128, 128, 2),
    "cfg4": GraphConfig("cfg4", 9_000_000, 1_000_000, 200_000_000, 0, 0, 128, 128, 2),
    "cfg5": GraphConfig("cfg5", 9_000_000, 1_000_000, 200_000_000, 90_000_000, 10_000_000,
                        128, 128, 2),
}


def replicated(name: str, world: int) -> GraphConfig:
    """Weak scaling: ``world`` copies' worth of nodes and edges in one global graph."""
    c = CONFIGS[name]
    if world == 1:
        return c
    return dataclasses.replace(c, name=f"{name}x{world}gpu", num_users=c.num_users * world,
                               num_posts=c.num_posts * world, num_engages=c.num_engages * world,
                               num_social=c.num_social * world,
                               num_post_post=c.num_post_post * world)


def scaled(name: str, factor: float) -> GraphConfig:
    """``name`` with every node and edge count multiplied by ``factor`` (>=1 node each)."""
    c = CONFIGS[name]
    f = lambda n: 0 if n == 0 else max(1, int(round(n * factor)))
    return dataclasses.replace(c, name=f"{name}x{factor:g}", num_users=f(c.num_users),
                               num_posts=f(c.num_posts), num_engages=f(c.num_engages),
                               num_social=f(c.num_social), num_post_post=f(c.num_post_post))


@dataclasses.dataclass
class SynthGraph:
    config: GraphConfig
    x_dict: Dict[str, torch.Tensor]
    edge_index_dict: Dict[EdgeType, torch.Tensor]

    @property
    def num_users(self) -> int:
        return self.config.num_users

    @property
    def num_posts(self) -> int:
        return self.config.num_posts

    def relations(self):
        return list(self.edge_index_dict.keys())

    def to(self, device) -> "SynthGraph":
        return SynthGraph(self.config, {k: v.to(device) for k, v in self.x_dict.items()},
                          {k: v.to(device) for k, v in self.edge_index_dict.items()})


def _zipf_cdf(n: int, s: float) -> np.ndarray:
    w = (np.arange(1, n + 1, dtype=np.float64)) ** (-s)
    c = np.cumsum(w)
    return c / c[-1]


def _zipf_sample_np(rng: np.random.Generator, n: int, size: int, s: float) -> np.ndarray:
    """Zipf-like ids over ``n`` items, ranks shuffled so the heavy ids are spread."""
    ranks = np.searchsorted(_zipf_cdf(n, s), rng.random(size), side="right")
    np.minimum(ranks, n - 1, out=ranks)
    perm = rng.permutation(n)
    return perm[ranks]


def _features_np(rng: np.random.Generator, n: int, d: int) -> np.ndarray:
    x = rng.standard_normal((n, d), dtype=np.float32)
    nrm = np.sqrt((x.astype(np.float64) ** 2).sum(1, keepdims=True))
    return (x / np.maximum(nrm, 1e-12)).astype(np.float32)


def make_graph(cfg: GraphConfig | str, device: str | torch.device = "cpu",
               device_gen: Optional[bool] = None, keep=None) -> SynthGraph:
    """Build the seeded graph.  CPU generation is numpy PCG64 (bit-reproducible everywhere).

    With a CUDA ``device`` and more than 50M edges (or ``device_gen=True``), the edges come from
    a counter-based generator (``_make_graph_counter``: edge e's endpoints are a hash of (seed,
    e), generated in chunks on the device, the same values on any device) and the features from
    a seeded torch generator (the same on every GPU): every rank of a multi-GPU run builds the
    identical global graph.  ``keep(edge_type, src, dst) -> bool mask`` (optional) filters each
    chunk as it is generated, so a rank can hold only its shard's edges
    (``parallel.shard_edge_filter``) without the global edge list ever existing on it; the kept
    edges keep their global order.  Only benches use this path; the parity tests' small graphs
    stay on numpy.
    """
    if isinstance(cfg, str):
        cfg = CONFIGS[cfg]
    dev = torch.device(device)
    big = dev.type == "cuda" and (cfg.num_engages + cfg.num_social) > 50_000_000
    if device_gen is not None:
        big = device_gen and dev.type == "cuda"
    if keep is not None and not big and dev.type == "cuda":
        raise ValueError("make_graph(keep=...) filters the counter-based device generator")
    if big or keep is not None:
        return _make_graph_counter(cfg, dev, keep)
    U, P = cfg.num_users, cfg.num_posts
    g = np.random.Generator(np.random.PCG64(GRAPH_SEED))
    if cfg.num_engages == 0:       # one engager per post (build_graph.py:390-394)
        eu = g.integers(0, U, size=P, dtype=np.int64)
        ep = np.arange(P, dtype=np.int64)
    else:
        eu = g.integers(0, U, size=cfg.num_engages, dtype=np.int64)
        ep = _zipf_sample_np(g, P, cfg.num_engages, cfg.zipf_s).astype(np.int64)
    eid: Dict[EdgeType, torch.Tensor] = {}
    if cfg.num_social:
        if cfg.num_engages == 0:   # toy: uniform follows, duplicates and self loops kept
            fs = g.integers(0, U, size=cfg.num_social, dtype=np.int64)
            ft = g.integers(0, U, size=cfg.num_social, dtype=np.int64)
        else:                      # power-law followees
            fs = g.integers(0, U, size=cfg.num_social, dtype=np.int64)
            ft = _zipf_sample_np(g, U, cfg.num_social, cfg.zipf_s).astype(np.int64)
        eid[SOCIAL] = torch.from_numpy(np.stack([fs, ft]))
    engage = torch.from_numpy(np.stack([eu, ep]))
    eid[ENGAGES] = engage
    eid[REV_ENGAGES] = engage.flip(0)           # train_gnn.py:142
    if cfg.num_post_post:
        ps = g.integers(0, P, size=cfg.num_post_post, dtype=np.int64)
        pt = _zipf_sample_np(g, P, cfg.num_post_post, cfg.zipf_s).astype(np.int64)
        eid[POST_POST] = torch.from_numpy(np.stack([ps, pt]))
    f = np.random.Generator(np.random.PCG64(FEAT_SEED))
    xu = torch.from_numpy(_features_np(f, U, cfg.dim))
    xp = torch.from_numpy(_features_np(f, P, cfg.dim))
    sg = SynthGraph(cfg, {"user": xu, "post": xp}, eid)
    return sg.to(dev) if dev.type != "cpu" else sg


# ----------------------------------------------------------------------------- counter-based
_GOLDEN = 0x9E3779B97F4A7C15 - (1 << 64)          # as int64 (wrapping arithmetic)
_M1 = 0xBF58476D1CE4E5B9 - (1 << 64)
_M2 = 0x94D049BB133111EB - (1 << 64)
GEN_CHUNK = 1 << 24                                 # edges generated per step


def _lsr(x: torch.Tensor, k: int) -> torch.Tensor:
    """Logical right shift of int64 (torch's >> is arithmetic)."""
    return (x >> k) & ((1 << (64 - k)) - 1)


def _hash64(stream: int, idx: torch.Tensor) -> torch.Tensor:
    """splitmix64 of (stream seed + idx * golden ratio): the counter-based draw of csrc's
    uniform_draw, in int64 torch ops (wrapping, bit-identical on CPU and GPU)."""
    x = idx * _GOLDEN + stream
    x = (x ^ _lsr(x, 30)) * _M1
    x = (x ^ _lsr(x, 27)) * _M2
    return x ^ _lsr(x, 31)


def _uniform_int(stream: int, idx: torch.Tensor, n: int) -> torch.Tensor:
    return (_lsr(_hash64(stream, idx), 32) * n) >> 32


def _uniform01(stream: int, idx: torch.Tensor) -> torch.Tensor:
    return _lsr(_hash64(stream, idx), 11).to(torch.float64) * (2.0 ** -53)


def _stream(name: str) -> int:
    """A fixed 63-bit seed per draw stream, derived from GRAPH_SEED."""
    h = GRAPH_SEED * 0x100000001B3 + sum((i + 1) * 131 ** i * ord(c) for i, c in enumerate(name))
    return h % (1 << 63)


def _make_graph_counter(cfg: GraphConfig, dev: torch.device, keep=None) -> SynthGraph:
    """Edges from counter-based draws (the distributions of the numpy path: uniform users,
    Zipf-like (rank+1)^-s post / followee ids over a shuffled rank order), chunk by chunk, each
    chunk filtered by ``keep``; features N(0,1) row-normalised from a seeded torch generator."""
    U, P = cfg.num_users, cfg.num_posts

    def perm(n, name):      # a random permutation of [0, n): argsort of hashed keys
        return torch.argsort(_hash64(_stream(name), torch.arange(n, device=dev)))

    cdf_cache = {}

    def zipf(n, name, idx):
        if n not in cdf_cache:
            cdf_cache[n] = (torch.from_numpy(_zipf_cdf(n, cfg.zipf_s)).to(dev), perm(n, name + "/perm"))
        cdf, pm = cdf_cache[n]
        r = torch.searchsorted(cdf, _uniform01(_stream(name), idx), right=True).clamp_(max=n - 1)
        return pm[r]

    def relation(et, n_edges, src_fn, dst_fn):
        parts = []
        for e0 in range(0, n_edges, GEN_CHUNK):
            idx = torch.arange(e0, min(e0 + GEN_CHUNK, n_edges), device=dev, dtype=torch.int64)
            src, dst = src_fn(idx), dst_fn(idx)
            if keep is not None:
                m = keep(et, src, dst)
                src, dst = src[m], dst[m]
            parts.append(torch.stack([src, dst]))
            del idx
        if not parts:
            return torch.empty(2, 0, dtype=torch.int64, device=dev)
        return torch.cat(parts, dim=1) if len(parts) > 1 else parts[0]

    eid: Dict[EdgeType, torch.Tensor] = {}
    if cfg.num_engages == 0:
        engage = relation(ENGAGES, P, lambda i: _uniform_int(_stream("eu"), i, U), lambda i: i)
    else:
        engage = relation(ENGAGES, cfg.num_engages, lambda i: _uniform_int(_stream("eu"), i, U),
                          lambda i: zipf(P, "ep", i))
    if cfg.num_social:
        eid[SOCIAL] = relation(SOCIAL, cfg.num_social, lambda i: _uniform_int(_stream("fs"), i, U),
                               lambda i: zipf(U, "ft", i))
    eid[ENGAGES] = engage
    eid[REV_ENGAGES] = engage.flip(0)           # train_gnn.py:142
    if cfg.num_post_post:
        eid[POST_POST] = relation(POST_POST, cfg.num_post_post,
                                  lambda i: _uniform_int(_stream("ps"), i, P),
                                  lambda i: zipf(P, "pt", i))
    gen = torch.Generator(device=dev)
    gen.manual_seed(FEAT_SEED)

    def feats(n):
        x = torch.randn(n, cfg.dim, generator=gen, device=dev)
        return torch.nn.functional.normalize(x, dim=1)

    return SynthGraph(cfg, {"user": feats(U), "post": feats(P)}, eid)


def negative_posts(num_posts: int, size: int, seed: int = NEG_SEED) -> torch.Tensor:
    """Injected negatives (train_gnn.py:272 draws them with torch.randint on the device)."""
    g = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(g.integers(0, num_posts, size=size, dtype=np.int64))


def interaction_weights(num_posts: int, seed: int = NEG_SEED + 10, qt_frac: float = 0.3) -> torch.Tensor:
    """Per-post interaction weight (train_gnn.py:226-237): QT -> 3.0 else 1.0, local post ids."""
    g = np.random.Generator(np.random.PCG64(seed))
    qt = g.random(num_posts) < qt_frac
    return torch.from_numpy(np.where(qt, 3.0, 1.0).astype(np.float32))


__all__ = ["CONFIGS", "GraphConfig", "SynthGraph", "make_graph", "scaled", "negative_posts",
           "interaction_weights", "ENGAGES", "REV_ENGAGES", "SOCIAL", "POST_POST"]
