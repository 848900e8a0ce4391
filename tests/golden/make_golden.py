"""Generate golden vectors for VectorQuantizerEMA by running the REFERENCE's
own vq_gnn_v2/vq.py (importable in the build container: torch + numpy only).

Run here only (the GPU box has no /root/reference):
    python tests/golden/make_golden.py
Each case is saved as tests/golden/vq_<name>.npz holding inputs, the
pre-state loaded into the reference module, its post-state, the returned
indices and the logging stash — data only, no reference source.
"""
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference/vq_gnn_v2"
OUT = os.path.dirname(os.path.abspath(__file__))


def load_ref():
    sys.path.insert(0, REF)
    import vq  # noqa: E402  (the reference module)
    return vq


def state_of(m):
    return dict(embedding=m._embedding.clone(), embedding_output=m._embedding_output.clone(),
                ema_cluster_size=m._ema_cluster_size.clone(), ema_w=m._ema_w.clone(),
                rm_f=m.batch_norm_feat.running_mean.clone(), rv_f=m.batch_norm_feat.running_var.clone(),
                rm_g=m.batch_norm_grad.running_mean.clone(), rv_g=m.batch_norm_grad.running_var.clone())


def make_case(vq, name, M, D, B, op, training=True, warm_up=True, grad_scale=(1.0, 1.0),
              momentum=0.1, calls=1, tie=False, seed=0, xscale=1.0, gscale=1e-3,
              cs_init=None, strided=False):
    torch.manual_seed(seed)
    m = vq.VectorQuantizerEMA(M, D, grad_normalize_scale=list(grad_scale),
                              warm_up_flag=warm_up, momentum=momentum)
    if cs_init is not None:
        m._ema_cluster_size.data.fill_(cs_init)
    if tie:  # duplicate codewords: exact ties must resolve to the first index
        m._embedding.data[M // 2:] = m._embedding.data[: M - M // 2]
    m.train(training)
    rec = {}
    for call in range(calls):
        pre = state_of(m)
        if strided:   # branch slices of wider activations, as the layers pass them
            X = (torch.randn(B, 3 * D) * xscale + 0.3).float()[:, D:2 * D]
            G = (torch.randn(B, 3 * D) * gscale).float()[:, 2 * D:3 * D]
        else:
            X = (torch.randn(B, D) * xscale + 0.3).float()
            G = (torch.randn(B, D) * gscale).float()
        err = ""
        idx = torch.full((B, 1), -1, dtype=torch.long)
        logs = {}
        pre_bn_inited = m.bn_inited
        try:
            if op == "feature_update":
                idx = m.feature_update(X)
            else:
                idx, _ = m.update(X, G)
                logs = dict(mean=m.mean.clone(), std=m.std.clone(),
                            feat_zero_rate=m.feat_zero_rate.clone(),
                            grad_zero_rate=m.grad_zero_rate.clone())
        except ValueError as e:
            err = str(e)
        post = state_of(m)
        p = f"c{call}_"
        rec[p + "X"] = X.contiguous().numpy()
        rec[p + "G"] = G.contiguous().numpy()
        rec[p + "idx"] = idx.numpy()[:, 0]
        rec[p + "error"] = np.array(err)
        rec[p + "bn_inited_pre"] = np.array(pre_bn_inited)
        for k, v in pre.items():
            rec[p + "pre_" + k] = v.numpy()
        for k, v in post.items():
            rec[p + "post_" + k] = v.numpy()
        for k, v in logs.items():
            rec[p + "log_" + k] = v.numpy()
        if err:
            break
    meta = dict(M=M, D=D, B=B, op=op, training=training, warm_up=warm_up,
                grad_scale=list(grad_scale), momentum=momentum, calls=calls,
                strided=strided, threads=torch.get_num_threads())
    rec["meta"] = np.array(repr(meta))
    np.savez_compressed(os.path.join(OUT, f"vq_{name}.npz"), **rec)
    print(name, {k: v.shape for k, v in rec.items() if k.endswith("idx")},
          "err=" + str(rec.get("c0_error")))


def main():
    torch.set_num_threads(8)
    vq = load_ref()
    make_case(vq, "fu_basic", 256, 4, 2000, "feature_update", calls=2)
    make_case(vq, "fu_eval", 256, 4, 1500, "feature_update", training=False)
    make_case(vq, "fu_bad_init", 64, 4, 40, "feature_update", warm_up=False)
    make_case(vq, "fu_m37", 37, 4, 1200, "feature_update", seed=3)
    make_case(vq, "fu_m1030", 1030, 4, 3000, "feature_update", seed=4)
    make_case(vq, "fu_tie", 64, 4, 800, "feature_update", tie=True, seed=5)
    make_case(vq, "fu_d2", 128, 2, 900, "feature_update", seed=6)
    make_case(vq, "up_basic", 256, 4, 2000, "update", calls=2, seed=7)
    make_case(vq, "up_scale", 128, 4, 1500, "update", grad_scale=(0.5, 1.0), momentum=0.2,
              calls=2, seed=8)
    make_case(vq, "up_scale0", 64, 4, 700, "update", grad_scale=(0.0, 1.0), seed=9)
    make_case(vq, "up_eval", 128, 4, 1000, "update", training=False, seed=10)
    make_case(vq, "up_tie", 64, 4, 600, "update", tie=True, seed=11)
    make_case(vq, "up_m4096", 4096, 4, 2500, "update", seed=12)
    make_case(vq, "up_nowarm", 32, 4, 3000, "update", warm_up=False, cs_init=1.0, seed=13)
    # strided inputs: ATen's non-contiguous BatchNorm path (cascade-sum mean)
    make_case(vq, "fu_strided", 256, 4, 5000, "feature_update", calls=2, seed=14, strided=True)
    make_case(vq, "fu_strided_eval", 128, 4, 1200, "feature_update", training=False, seed=15,
              strided=True)
    make_case(vq, "up_strided", 256, 4, 4500, "update", calls=2, seed=16, strided=True)
    make_case(vq, "up_strided_m1024", 1024, 4, 10000, "update", seed=17, strided=True,
              xscale=2.0)
    make_case(vq, "up_strided_scale", 128, 4, 1500, "update", grad_scale=(0.5, 1.0),
              momentum=0.2, calls=2, seed=18, strided=True)
    make_case(vq, "up_strided_eval", 128, 4, 1000, "update", training=False, seed=19,
              strided=True)


if __name__ == "__main__":
    main()
