"""Plain-torch stand-ins for the compute ops of truth_recommendation_gnn_amd.parallel — TEST
ONLY: lets the world_size-2 gloo tests check the partitioning and collective logic on CPU (the
HIP kernels themselves are checked by tests/test_gpu_parity.py)."""
import torch
import torch.nn.functional as F

from oracle import sage_ref


def _torch_fused_weights(convs, msgs, x_dict):
    """[w_1 W_l,1 | ... | w_R W_l,R | sum_r w_r W_r,r] and sum_r w_r b_r with torch ops
    (autograd-tracked): the CPU stand-in of nn._fused_weights."""
    w_ls, w_root, b = [], None, None
    for name, et, wt in msgs:
        conv = convs[name]
        conv.materialize(x_dict[et[0]].shape[1], x_dict[et[2]].shape[1])
        scale = (lambda t: t) if wt == 1.0 else (lambda t: t * wt)
        w_ls.append(scale(conv.lin_l.weight))
        if conv.lin_r is not None:
            r = scale(conv.lin_r.weight)
            w_root = r if w_root is None else w_root + r
        if conv.lin_l.bias is not None:
            bb = scale(conv.lin_l.bias)
            b = bb if b is None else b + bb
    parts = w_ls + ([w_root] if w_root is not None else [])
    return torch.cat(parts, dim=1), b


def _torch_grads_to_params(convs, msgs, dW, db):
    """The adjoint of _torch_fused_weights, accumulated into each parameter's .grad."""
    def acc(p, g):
        if p.grad is None:
            p.grad = g
        else:
            p.grad.add_(g)
    off = 0
    for name, _, wt in msgs:
        conv = convs[name]
        k = conv.lin_l.weight.shape[1]
        acc(conv.lin_l.weight, (dW[:, off:off + k] * wt).contiguous())
        if conv.lin_l.bias is not None and db is not None:
            acc(conv.lin_l.bias, db * wt)
        off += k
    root = dW[:, off:]
    for name, _, wt in msgs:
        conv = convs[name]
        if conv.lin_r is not None:
            acc(conv.lin_r.weight, (root * wt).contiguous())


class TorchImpl:
    fused_weights = staticmethod(_torch_fused_weights)
    grads_to_params = staticmethod(_torch_grads_to_params)

    def relation(self, edge_index, n_src, n_dst):
        return (edge_index, n_src, n_dst)

    def edge_weights_fwd(self, rel, w_dst):
        return w_dst[rel[0][1]]          # per COO edge

    def edge_weights_bwd(self, rel, w_dst):
        return w_dst[rel[0][1]]

    @staticmethod
    def mean_gather(x, rel):
        ei, _, n_dst = rel
        out = sage_ref.mean_aggregate(x, ei, n_dst)
        if ei.shape[1] == 0:
            # connected to x, as the HIP op is (its backward returns a zero gradient): every
            # rank's autograd graph then has the same shape, so the collective adjoints run in
            # the same order everywhere
            out = out + x.sum() * 0.0
        return out

    @staticmethod
    def weighted_gather(x, rel, w_fwd, w_bwd):
        ei, _, n_dst = rel
        out = torch.zeros(n_dst, x.shape[1], dtype=x.dtype)
        return out.index_add(0, ei[1], x[ei[0]] * w_fwd[:, None])

    @staticmethod
    def fused_linear(segs, w, b, relu, add=None):
        y = F.linear(torch.cat(segs, 1), w, b)
        if add is not None:
            y = y + add
        return F.relu(y) if relu else y

    @staticmethod
    def edge_bce_loss(U, P, pos, neg, n_total, cscale, neg_order="edge", ready=None):
        if ready is not None:
            ready()
        u = U[pos[0]]
        s_pos = (u * P[pos[1]]).sum(1)
        s_neg = (u * P[neg]).sum(1)
        return (cscale * F.softplus(-s_pos).sum() + F.softplus(s_neg).sum()) / n_total

    # raw forms for UserShard.step's explicit schedule
    gather_mean_raw = mean_gather

    @staticmethod
    def weighted_gather_raw(x, rel, w_fwd, row_w=None):
        ei, _, n_dst = rel
        return torch.zeros(n_dst, x.shape[1], dtype=x.dtype).index_add(0, ei[1],
                                                                        x[ei[0]] * w_fwd[:, None])

    @staticmethod
    def scatter_mean_bwd_raw(g, rel, out=None):
        ei, n_src, n_dst = rel
        deg = torch.bincount(ei[1], minlength=n_dst).clamp(min=1).to(g.dtype)
        if out is None:
            out = torch.zeros(n_src, g.shape[1], dtype=g.dtype)
        return out.index_add_(0, ei[0], g[ei[1]] / deg[ei[1]][:, None])

    @staticmethod
    def weighted_scatter_bwd_raw(g, rel, w_bwd, out=None):
        ei, n_src, _ = rel
        if out is None:
            out = torch.zeros(n_src, g.shape[1], dtype=g.dtype)
        return out.index_add_(0, ei[0], g[ei[1]] * w_bwd[:, None])

    linear_fwd_raw = fused_linear

    @staticmethod
    def linear_bwd_raw(segs, w, dout, out_act, dxs, need_w, need_b, dz_out=None):
        dz = dout * (out_act > 0) if out_act is not None else dout
        if dz_out is not None:
            dz_out.copy_(dz)
        x = torch.cat(segs, 1)
        dx = dz @ w
        o = 0
        for s, t in zip(segs, dxs):
            if t is not None:
                t.copy_(dx[:, o:o + s.shape[1]])
            o += s.shape[1]
        return (dz.T @ x if need_w else None), (dz.sum(0) if need_b else None)

    def edge_bce_loss_raw(self, U, P, pos, neg, n_total, cscale, neg_order="edge", ready=None,
                          on_dP=None, p_chunks=None):
        for _, _, rdy in (p_chunks or ()):
            if rdy is not None:
                rdy()
        if ready is not None:
            ready()
        U2, P2 = U.detach().requires_grad_(), P.detach().requires_grad_()
        with torch.enable_grad():
            loss = self.edge_bce_loss(U2, P2, pos, neg, n_total, cscale)
            dU, dP = torch.autograd.grad(loss, (U2, P2))
        if on_dP is not None:
            on_dP(dP)
        return loss.detach(), dU, dP
