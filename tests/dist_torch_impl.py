"""Plain-torch stand-ins for the compute ops of truth_recommendation_gnn_amd.parallel — TEST
ONLY: lets the world_size-2 gloo tests check the partitioning and collective logic on CPU (the
HIP kernels themselves are checked by tests/test_gpu_parity.py)."""
import torch
import torch.nn.functional as F

from oracle import sage_ref


class TorchImpl:
    def relation(self, edge_index, n_src, n_dst):
        return (edge_index, n_src, n_dst)

    def edge_weights_fwd(self, rel, w_dst):
        return w_dst[rel[0][1]]          # per COO edge

    def edge_weights_bwd(self, rel, w_dst):
        return w_dst[rel[0][1]]

    @staticmethod
    def mean_gather(x, rel):
        ei, _, n_dst = rel
        return sage_ref.mean_aggregate(x, ei, n_dst)

    @staticmethod
    def weighted_gather(x, rel, w_fwd, w_bwd):
        ei, _, n_dst = rel
        out = torch.zeros(n_dst, x.shape[1], dtype=x.dtype)
        return out.index_add(0, ei[1], x[ei[0]] * w_fwd[:, None])

    @staticmethod
    def fused_linear(segs, w, b, relu):
        y = F.linear(torch.cat(segs, 1), w, b)
        return F.relu(y) if relu else y

    @staticmethod
    def edge_bce_loss(U, P, pos, neg, n_total, cscale, neg_order="edge", ready=None):
        if ready is not None:
            ready()
        u = U[pos[0]]
        s_pos = (u * P[pos[1]]).sum(1)
        s_neg = (u * P[neg]).sum(1)
        return (cscale * F.softplus(-s_pos).sum() + F.softplus(s_neg).sum()) / n_total
