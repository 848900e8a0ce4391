"""Drop-in ``LowRankGNNBlock`` / ``LowRankGNNLayer`` / ``LowRankGNN``
(reference: vq_gnn_v2/models.py).

Same constructors, submodule names, buffer names and return tuples.  What is
different is where the work happens:

* the nb per-branch VQ steps of a layer (models.py:161-171) are ONE batched
  launch sequence over a packed ``VQBank`` (vq.py here);
* ``c_indices`` of all blocks of a layer live in one node-major int16 array
  [N, nb]; each block's ``c_indices`` is the column view ``codes[:, i]``;
* the per-branch codebook gathers (models.py:168-173) are one codeword-gather
  launch over all branches, and ``torch.cat`` + ``self.conv(x_input, adj)``
  (models.py:174-179) one two-source SpMM launch (convs.py here).

Reference behaviour that is kept on purpose: the backward
hooks registered at models.py:181-185 never fire in v2 (they sit on an
unconsumed view), so the codebooks move only through ``init`` /
``feature_update``.  ``vq_update_in_backward=True`` opts in to the update the
hook was meant to perform (the v1 semantics), batched over branches.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import kernels
from .convs import CodebookInput, OurGCNConv, _VQHook
from .sparse import as_csr
from .vq import VectorQuantizerEMA, VQBank


class LowRankGNNBlock(torch.nn.Module):
    """Reference: models.py:11-63.  Holds one branch's ``vq`` and its
    ``c_indices`` (a column view of the layer's packed codes)."""

    def __init__(self, in_channels, hidden_channels, num_M, num_D, num_N, num_branch, cluster,
                 kmeans_iter, EMA_flag, kmeans_init, use_gcn, commitment_cost,
                 grad_normalize_scale, hook_flag, warm_up_flag, momentum, conv_type,
                 transformer_flag, _bank=None, _codes=None, _branch=0):
        super().__init__()
        self.num_M, self.num_D, self.num_N, self.EMA_flag = num_M, num_D, num_N, EMA_flag
        self.commitment_cost = commitment_cost
        self.hook_flag = hook_flag
        self.grad_normalize_scale = grad_normalize_scale
        self.conv_type = conv_type
        self.transformer_flag = transformer_flag
        self._branch = int(_branch)
        c = torch.randint(0, self.num_M, (self.num_N,), dtype=torch.short)  # models.py:27
        if _codes is None:
            self.register_buffer("_own_codes", c.view(-1, 1), persistent=False)
            self.__dict__["_codes_owner"] = None
        else:
            self.__dict__["_codes_owner"] = _codes
            _codes()[:, self._branch].copy_(c)
        if _bank is not None:
            _bank.init_branch(self._branch)
        self.vq = VectorQuantizerEMA(self.num_M, self.num_D, commitment_cost=self.commitment_cost,
                                     grad_normalize_scale=grad_normalize_scale,
                                     warm_up_flag=warm_up_flag, momentum=momentum,
                                     add_flag=False, _bank=_bank, _branch=self._branch)
        self.kmeans_init = kmeans_init
        self.grad_kmeans_init = kmeans_init
        self.inited = False
        self.X_B = None
        self.batch_indices = None
        self.__dict__["_vq_backward_error"] = None

    @property
    def c_indices(self):
        owner = self.__dict__.get("_codes_owner")
        if owner is None:
            return self._own_codes.data[:, 0]
        return owner()[:, self._branch]

    @property
    def vq_backward_error(self):
        v = self.__dict__.get("_vq_backward_error")
        return None if v is None else float(v.item())

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        destination[prefix + "c_indices"] = self.c_indices.detach().clone()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        if prefix + "c_indices" in state_dict:
            with torch.no_grad():
                self.c_indices.copy_(state_dict[prefix + "c_indices"])
        elif strict:
            missing_keys.append(prefix + "c_indices")

    def hook(self, grad):                                          # models.py:39-56
        encoding_indices, _ = self.vq.update(self.X_B, grad)
        self.c_indices[self.batch_indices] = encoding_indices.squeeze().to(torch.short)
        X_B_diff = self.X_B - self.vq.get_codebook()[encoding_indices.squeeze()]
        self.__dict__["_vq_backward_error"] = torch.norm(X_B_diff, dim=1).mean()
        return grad

    def init(self, X_B, batch_indices):                            # models.py:61-63
        encoding_indices = self.vq.feature_update(X_B)
        self.c_indices[batch_indices] = encoding_indices.squeeze().to(torch.short)


class LowRankGNNLayer(torch.nn.Module):
    """Reference: models.py:66-231."""

    def __init__(self, in_channels, out_channels, dropout, num_M, num_D, num_N, num_branch,
                 cluster, ln_para, no_second_fc, kmeans_iter, EMA_flag, split, kmeans_init,
                 dropbranch, skip, use_gcn, commitment_cost, grad_normalize_scale, hook,
                 weight_ahead, warm_up_flag, momentum, conv_type, transformer_flag,
                 vq_update_in_backward=False):
        super().__init__()
        self.weight_ahead = weight_ahead
        if self.weight_ahead:
            if out_channels % num_D != 0:
                raise ValueError('Cannot fully split')
            self.num_branch = int(out_channels / num_D)
        else:
            if in_channels % num_D != 0:
                raise ValueError('Cannot fully split')
            self.num_branch = int(in_channels / num_D)
        if in_channels != self.num_branch * num_D:
            raise ValueError('Cannot fully split')   # the reference fails later in torch.cat

        self.out_channels = out_channels
        self.no_second_fc = no_second_fc
        self.EMA_flag = EMA_flag
        self.split = split
        self.num_D = num_D
        self.dropbranch = dropbranch
        self.skip = skip
        self.conv_type = conv_type
        self.transformer_flag = transformer_flag
        self.num_M = num_M
        self.num_N = num_N
        self.vq_update_in_backward = vq_update_in_backward

        if self.conv_type != 'GAT':
            self.conv = OurGCNConv(in_channels, in_channels, normalize=False)
        else:
            from .convs_gat import OurGATConv
            self.conv = OurGATConv(in_channels + 1, in_channels + 1, bias=False,
                                   add_self_loops=False)

        nb = self.num_branch
        self._bank = VQBank(nb, num_M, num_D, 0.99, 1e-24, grad_normalize_scale, warm_up_flag,
                            momentum)
        self.register_buffer("_codes", torch.empty(num_N, nb, dtype=torch.int16),
                             persistent=False)
        codes_getter = lambda: self._codes  # noqa: E731  (always the current buffer)
        self.linear_k, self.linear_v = torch.nn.ModuleList(), torch.nn.ModuleList()
        self.gnn_block, self.transformer_block = torch.nn.ModuleList(), torch.nn.ModuleList()
        if transformer_flag:
            raise NotImplementedError("transformer_flag: the reference's use of it is commented "
                                      "out (models.py:206-226)")
        for i in range(nb):
            if no_second_fc:
                self.gnn_block.append(LowRankGNNBlock(
                    None, None, num_M, num_D, num_N, nb, cluster, kmeans_iter, EMA_flag,
                    kmeans_init, use_gcn, commitment_cost, grad_normalize_scale, hook,
                    warm_up_flag, momentum, conv_type, False,
                    _bank=self._bank, _codes=codes_getter, _branch=i))
            else:
                raise ValueError('second fc not studied')

        if self.skip:
            self.linear_skip = torch.nn.Linear(in_channels, out_channels)
        self.gnn_transform = torch.nn.Linear(in_channels, out_channels)
        self.batch_norm = torch.nn.BatchNorm1d(out_channels, affine=False)
        if self.conv_type == 'SAGE':
            self.fc_sage = torch.nn.Linear(in_channels, out_channels)

    # ------------------------------------------------------------------ #
    def _batched_init(self, x, batch_idx):
        """All branches' LowRankGNNBlock.init (models.py:165-166) in one launch
        sequence: feature_update + c_indices scatter."""
        self._bank.feature_update(x, 0, self.num_branch, self.training, codes=self._codes,
                                  batch_idx=batch_idx)

    def _backward_vq_update(self, x_detached, grad_B, batch_idx):
        """The v1 hook semantics (models.py:39-56) for all branches at once."""
        self._bank.update(x_detached, grad_B, 0, self.num_branch, True, codes=self._codes,
                          batch_idx=batch_idx)

    def forward(self, x, batch_A, warm_up_rate, unlabeled):
        errors, X_B_norms, quantized_norms = [], [], []
        losses, info_backwards = 0, 0
        hookeds = []

        if self.training and self.dropbranch > 0:
            raise NotImplementedError(
                "dropbranch > 0: the reference's torch.cat at models.py:174 fails for a "
                "partial branch set")
        branch_idx = range(self.num_branch)

        batch_idx, subset, adj = batch_A
        adj = as_csr(adj)
        B = x.shape[0]
        D = self.num_D

        x_det = x.detach()
        for i in branch_idx:
            blk = self.gnn_block[i]
            blk.X_B = x_det[:, D * i:D * (i + 1)]
            blk.batch_indices = batch_idx
        need = [i for i in branch_idx if (not self.gnn_block[i].inited) or unlabeled]
        if len(need) == self.num_branch:
            xc = x_det if x_det.stride(1) == 1 else x_det.contiguous()
            self._batched_init(xc, batch_idx)
        else:
            for i in need:
                self.gnn_block[i].init(x_det[:, D * i:D * (i + 1)], batch_idx)

        # x_first_order (models.py:168-173): codeword feature halves of B' --
        # materialised for GAT; GCN / SAGE read them from the codebook inside
        # the SpMM where the shape allows (CodebookInput)
        x_first = None
        if self.conv_type == 'GAT':
            x_first, _ = kernels.gather_codewords(subset, B, self._codes, self._bank.emb_out, D)

        hook = None
        if self.vq_update_in_backward and self.training and not unlabeled and \
                all(self.gnn_block[i].inited for i in branch_idx):
            hook = _VQHook(self, x_det, batch_idx)

        if self.conv_type == 'GAT':
            x_output = self.conv.fused_forward(x, adj, x_first, B, hook)
        else:
            x_output = self.conv(CodebookInput(x, subset, self._codes, self._bank.emb_out, D),
                                 adj, _hook=hook)
        # multi-GPU: the other ranks' new codes were exchanged behind the
        # gather + aggregation; land them before anything reads c_indices again
        self._bank.sync_codes()

        for _ in branch_idx:
            errors.append(0)
            X_B_norms.append(0)
            quantized_norms.append(0)

        # info_backward (models.py:198): sum(out[B:] * grad half of the codewords)
        grad_first_order, _ = kernels.gather_codewords(subset, B, self._codes,
                                                       self._bank.emb_out, D, col_offset=D)
        info_backward = torch.sum(x_output[B:] * grad_first_order * warm_up_rate)
        if self.training:
            info_backwards += info_backward

        x_output = self.gnn_transform(x_output[:B])
        if self.conv_type == 'SAGE':
            x_output = x_output + self.fc_sage(x)
        if self.skip:
            x_output = x_output + self.linear_skip(x)
        return x_output, errors, X_B_norms, quantized_norms, losses, info_backwards, hookeds


class LowRankGNN(torch.nn.Module):
    """Reference: models.py:234-374."""

    def __init__(self, in_channels, hidden_channels, out_channels, num_layers, dropout, num_M,
                 num_D, num_N, num_branch=0, cluster='vq', ln_para=True, no_second_fc=False,
                 kmeans_iter=100, EMA_flag=True, split=True, kmeans_init=False, dropbranch=0,
                 skip=True, use_gcn=False, commitment_cost=0.5, grad_scale=(1, 1), act='relu',
                 weight_ahead=False, bn_flag=False, warm_up_flag=False, momentum=0.1,
                 conv_type='GCN', transformer_flag=False, alpha_dropout_flag=False,
                 vq_update_in_backward=False):
        super().__init__()
        self.num_layers = num_layers
        self.skip = skip
        self.dropout = dropout
        self.bn_flag = bn_flag
        self.alpha_dropout_flag = alpha_dropout_flag
        if self.alpha_dropout_flag:
            self.alpha_dropout = torch.nn.AlphaDropout(p=self.dropout)

        common = dict(num_branch=num_branch, cluster=cluster, ln_para=ln_para,
                      no_second_fc=no_second_fc, kmeans_iter=kmeans_iter, EMA_flag=EMA_flag,
                      split=split, kmeans_init=kmeans_init, skip=skip, use_gcn=use_gcn,
                      commitment_cost=commitment_cost, grad_normalize_scale=grad_scale,
                      hook=True, weight_ahead=weight_ahead, warm_up_flag=warm_up_flag,
                      momentum=momentum, conv_type=conv_type, transformer_flag=transformer_flag,
                      vq_update_in_backward=vq_update_in_backward)
        self.convs, self.batch_norms = torch.nn.ModuleList(), torch.nn.ModuleList()
        self.convs.append(LowRankGNNLayer(in_channels, hidden_channels, dropout, num_M, num_D,
                                          num_N, dropbranch=0, **common))
        self.batch_norms.append(torch.nn.BatchNorm1d(hidden_channels, affine=False))
        for _ in range(num_layers - 2):
            self.convs.append(LowRankGNNLayer(hidden_channels, hidden_channels, dropout, num_M,
                                              num_D, num_N, dropbranch=dropbranch, **common))
            self.batch_norms.append(torch.nn.BatchNorm1d(hidden_channels, affine=False))
        self.convs.append(LowRankGNNLayer(hidden_channels, out_channels, dropout, num_M, num_D,
                                          num_N, dropbranch=dropbranch, **common))

        self.transform = torch.nn.Linear(out_channels, out_channels)
        self.ln = torch.nn.LayerNorm(hidden_channels, elementwise_affine=False)
        if act == 'relu':
            self.act_f = F.relu
        elif act == 'elu':
            self.act_f = F.elu
        elif act == 'leaky_gelu':
            self.act_f = lambda x: 0.1 * x + 0.9 * F.gelu(x)
        else:
            raise ValueError('Activation not supported!')

    def forward(self, batch, warm_up_rate=1, unlabeled=False):       # models.py:308-348
        losses_full, info_backwards_full = 0, 0
        errors_full, X_B_norms_full, quantized_norms_full = [], [], []
        x, batch_A = batch
        for i, conv in enumerate(self.convs[:-1]):
            x, errors, X_B_norms, quantized_norms, losses, info_backwards, _ = \
                conv(x, batch_A, warm_up_rate, unlabeled)
            if self.bn_flag:
                x = self.batch_norms[i](x)
            x = self.act_f(x)
            if self.alpha_dropout_flag:
                x = self.alpha_dropout(x)
            else:
                x = F.dropout(x, p=self.dropout, training=self.training)
            losses_full += losses
            info_backwards_full += info_backwards
            errors_full.append(errors)
            X_B_norms_full.append(X_B_norms)
            quantized_norms_full.append(quantized_norms)
        x, errors, X_B_norms, quantized_norms, losses, info_backwards, _ = \
            self.convs[-1](x, batch_A, warm_up_rate, unlabeled)
        losses_full += losses
        info_backwards_full += info_backwards
        errors_full.append(errors)
        X_B_norms_full.append(X_B_norms)
        quantized_norms_full.append(quantized_norms)
        self.errors, self.X_B_norms, self.quantized_norms = \
            errors_full, X_B_norms_full, quantized_norms_full
        return x, losses_full, info_backwards_full

    def inference(self, x, A):                                       # models.py:350-367
        # Broken in the reference (gnn_block[0].conv does not exist in v2);
        # kept with the same AttributeError so callers see identical behaviour.
        raise AttributeError("'LowRankGNNBlock' object has no attribute 'conv'")

    def init(self, batch, layer_idx):                                # models.py:370-374
        x, batch_A = batch
        for i, conv in enumerate(self.convs[:layer_idx]):
            x, _, _, _, _, _, _ = conv(x, batch_A, 1, False)
            x = self.act_f(x)
