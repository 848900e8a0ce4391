"""3-layer model total: one training step of LowRankGNN on the
arxiv-shaped batch (3 x LowRankGNNLayer, F = 128/128/128 -> 40, M = 256,
D = 4; main_node.py's step: forward, cross entropy + info_backward,
backward, RMSprop step), timed on the GPU with the inputs resident.

Two forms:
  v2     the reference's v2 training step (the VQ hooks never fire,
         models.py:181-185): per layer gather + SpMM forward, A^T backward;
  hook   vq_update_in_backward=True (v1 semantics): each
         layer's backward also runs the batched VQ update (assign + EMA) on
         dOut[:B];
  hook_overlap  the same with that update on a side stream beside the
         layer's A^T product (VQGNN_HOOK_OVERLAP=1).
Prints one JSON line per form: ms per step, model edges/s = 3 * nnz / step.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import vqgnn_pkg  # noqa: E402

vqgnn_pkg.load()
from vq_gnn_amd.graph import CONFIGS, batch_to_device, make_batch  # noqa: E402
from vq_gnn_amd.models import LowRankGNN  # noqa: E402


def run(form, steps, warmup, cfg_name):
    cfg = CONFIGS[cfg_name]
    dev = torch.device("cuda:0")
    g, _, b = make_batch(cfg)
    F, M = cfg["F"], cfg["M"]
    torch.manual_seed(0)
    model = LowRankGNN(F, F, 40, 3, 0.0, M, 4, g.N, no_second_fc=True, skip=True,
                       grad_scale=[1, 1], act='relu', bn_flag=True, warm_up_flag=True,
                       conv_type=cfg["conv"],
                       vq_update_in_backward=form.startswith("hook")).to(dev)
    os.environ["VQGNN_HOOK_OVERLAP"] = "1" if form == "hook_overlap" else "0"
    batch_A = batch_to_device(b, dev)
    x = torch.randn(b.B, F, device=dev)
    y = torch.randint(0, 40, (b.B,), device=dev)
    model.train()
    with torch.no_grad():
        for layer_idx in range(1, 4):                 # main_node.py:90-95 init pass
            model.init((x, batch_A), layer_idx)
    for layer in model.convs:
        for blk in layer.gnn_block:
            blk.inited = True
    opt = torch.optim.RMSprop(model.parameters(), lr=1e-3, alpha=0.99)

    def step():
        opt.zero_grad()
        out, _, info_b = model((x, batch_A), 1.0)
        loss = torch.nn.functional.cross_entropy(out, y) + info_b
        loss.backward()
        opt.step()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return dict(metric="3-layer model training step", form=form, config=cfg_name,
                ms_per_step=dt * 1e3, model_edges_per_s=3 * b.nnz / dt, B=b.B, n=b.n,
                nnz=b.nnz, F=F, M=M, layers=3, steps=steps, warmup=warmup)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="arxiv_gcn")
    p.add_argument("--forms", default="v2,hook,hook_overlap")
    a = p.parse_args()
    for form in a.forms.split(","):
        print(json.dumps(run(form, a.steps, a.warmup, a.config)), flush=True)


if __name__ == "__main__":
    main()
