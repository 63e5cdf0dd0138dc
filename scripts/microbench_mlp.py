"""Micro-benchmark of the fused MLP train-step kernel on one GPU (eager and
hipGraph-captured), plus the same step in stock PyTorch for comparison."""
import argparse
import json
import time

import torch

from distributed_training_amd.ops import mlp_fused as mf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--in-dim", type=int, default=20)
    ap.add_argument("--out-dim", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--own", type=int, default=4)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--unroll", type=int, default=32)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lay = mf.make_layout(args.in_dim, args.hidden, args.out_dim)
    N = 2048
    X = torch.rand(N, args.in_dim, device=dev)
    T = torch.rand(N, args.out_dim, device=dev)
    ring = torch.randint(0, N, (64, args.batch), dtype=torch.int32, device=dev)
    cursor = torch.zeros(1, dtype=torch.int32, device=dev)
    stage = mf.make_stage(dev)
    loss = torch.zeros(64, device=dev)
    P = [torch.randn(lay.total, device=dev) * 0.05 for _ in range(2)]
    G = [torch.zeros(lay.total, device=dev) for _ in range(2)]
    sgd = {"lr": 1e-3}

    def step(i):
        a, b = i % 2, (i + 1) % 2
        mf.fused_step(X, T, ring, cursor, stage, loss, P[a], P[b], G[b], G[a], None, None, lay, args.batch,
                      args.own, "relu", "mse", True, 1.0, sgd, 1.0, False, parity=a, gather_self=False)

    for i in range(50):
        step(i)
    torch.cuda.synchronize()
    stamps = torch.zeros(8 * 64, dtype=torch.int64, device=dev)
    phase_us = []
    for rep in range(20):
        mf.fused_step(X, T, ring, cursor, stage, loss, P[0], P[1], G[1], G[0], None, None, lay, args.batch,
                      args.own, "relu", "mse", True, 1.0, sgd, 1.0, False, dbg_stamps=stamps, parity=0,
                      gather_self=False)
        torch.cuda.synchronize()
        st = stamps.view(64, 8).cpu()
        nwg = (args.hidden // 32 + args.own - 1) // args.own
        d = (st[:nwg, 1:5] - st[:nwg, 0:4]).float().mean(0) / 100.0  # 100 MHz ticks -> us
        tot = (st[:nwg, 4].max() - st[:nwg, 0].min()).item() / 100.0
        d[3] = (st[0, 4] - st[0, 3]).item() / 100.0  # WG0 tail
        clk = ((st[:nwg, 6] - st[:nwg, 5]).float() / (st[:nwg, 4] - st[:nwg, 0]).float() * 100.0).mean().item()
        phase_us.append(d.tolist() + [tot, clk])
    phase_us = torch.tensor(phase_us).median(0).values.tolist()
    t0 = time.perf_counter()
    for i in range(args.iters):
        step(i)
    torch.cuda.synchronize()
    eager_us = (time.perf_counter() - t0) / args.iters * 1e6

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for i in range(4):
            step(i)
        torch.cuda.current_stream().synchronize()
        with torch.cuda.graph(g, stream=s):
            for i in range(args.unroll):
                step(i)
    torch.cuda.synchronize()
    reps = max(1, args.iters // args.unroll)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    graph_us = (time.perf_counter() - t0) / (reps * args.unroll) * 1e6

    # stock torch reference step (eager, bf16 autocast, same shapes)
    model = torch.nn.Sequential(torch.nn.Linear(args.in_dim, args.hidden), torch.nn.ReLU(),
                                torch.nn.Linear(args.hidden, args.out_dim)).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)
    Xb = X[:args.batch]
    Tb = T[:args.batch]

    def tstep():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = model(Xb)
        l = torch.nn.functional.mse_loss(y.float(), Tb)
        l.backward()
        opt.step()

    for _ in range(20):
        tstep()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(500):
        tstep()
    torch.cuda.synchronize()
    torch_us = (time.perf_counter() - t0) / 500 * 1e6
    print(json.dumps({"hidden": args.hidden, "batch": args.batch, "own_tiles": args.own, "eager_us": eager_us,
                      "graph_us_per_step": graph_us, "torch_eager_us": torch_us,
                      "phase_us[p0,p1,p2,p3,total,clockMHz]": [round(x, 2) for x in phase_us]}))


if __name__ == "__main__":
    main()
