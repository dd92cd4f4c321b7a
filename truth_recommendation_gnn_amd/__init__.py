"""hgnn on MI355X: the hetero SAGE message-passing hot path of ramkp990/Truth_Recommendation_GNN,
rebuilt as hand-written gfx950 HIP kernels behind a C ABI (``include/hgnn.h``), with the
reference's PyG-style Python surface (``SAGEConv``, ``HeteroData``, ``WeightedRGCN``).
"""
from .graph import HeteroData, RelationCSR, relation_csr, CSR_CACHE  # noqa: F401
from .nn import SAGEConv, WeightedRGCN, WeightedRGCNAuthor, HeteroSAGE  # noqa: F401
from . import ops, synth  # noqa: F401
from .metrics import evaluate, recommend  # noqa: F401

__version__ = "0.1.0"
