"""One-shot peer-memory all-reduce (csrc/p2p_allreduce.hip), exercised by two
processes sharing the box's single GPU: the IPC export/open, push, flag
protocol, parity double-buffering, graph replay and the timeout path are the
same code as across xGMI peers (only the link differs)."""
import pytest
import torch

from dist_utils import run_gloo

pytestmark = pytest.mark.gpu


def _make(rank, ws, tag, **kw):
    import torch.distributed as dist

    from distributed_training_amd.parallel.p2p import P2PAllReduce

    store = dist.distributed_c10d._get_default_store()
    return P2PAllReduce(rank, ws, torch.device("cuda", 0), store, tag=tag, **kw)


def _expected(xs_local, ws):
    import torch.distributed as dist

    cpu = xs_local.cpu()
    parts = [torch.empty_like(cpu) for _ in range(ws)]
    dist.all_gather(parts, cpu)
    acc = torch.zeros_like(cpu)
    for p in parts:  # rank order, like the kernel
        acc += p
    return acc


def _worker(rank, ws, protocol):
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    p2p = _make(rank, ws, "t1", protocol=protocol)
    g = torch.Generator(device="cpu").manual_seed(10 + rank)
    # sizes: scalar tail, one workgroup, several, many (64 WG cap), slot capacity
    for n in (1, 5, 2048, 4099, 11280, 70001, 262144):
        for it in range(3):  # both parities
            x = torch.randn(n, generator=g).to(dev)
            want = _expected(x, ws)
            p2p.all_reduce(x, 1.0)
            torch.cuda.synchronize()
            p2p.check()
            assert torch.equal(x.cpu(), want), (n, it, (x.cpu() - want).abs().max())
    # averaging scale + many back-to-back launches without host sync
    xs = [torch.full((11280,), float(rank + 1 + i), device=dev) for i in range(50)]
    for x in xs:
        p2p.all_reduce(x, 1.0 / ws)
    torch.cuda.synchronize()
    p2p.check()
    for i, x in enumerate(xs):
        want = sum(r + 1 + i for r in range(ws)) / ws
        assert torch.allclose(x, torch.full_like(x, want)), i
    # hipGraph capture + replay (epochs advance on the device)
    buf = torch.zeros(11280, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            for _ in range(4):
                buf.add_(1.0)
                p2p.all_reduce(buf, 1.0, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for rep in range(3):
        buf.fill_(float(rank))
        graph.replay()
        torch.cuda.synchronize()
        p2p.check()
        # each captured step: b_r += 1, then every rank holds sum_r b_r
        b = [float(r) for r in range(ws)]
        for _ in range(4):
            tot = sum(x + 1.0 for x in b)
            b = [tot] * ws
        assert torch.allclose(buf, torch.full_like(buf, b[rank])), (rep, buf[0].item(), b[rank])
    p2p.destroy()


def _timeout_worker(rank, ws, protocol):
    import torch.distributed as dist

    torch.cuda.set_device(0)
    p2p = _make(rank, ws, "t2", timeout_iters=1 << 12, protocol=protocol)
    x = torch.ones(1000, device="cuda")
    if rank == 0:  # the peer never joins: the kernel must give up and flag the error
        p2p.all_reduce(x, 1.0)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="timed out"):
            p2p.check()
        with pytest.raises(RuntimeError, match="timed out"):  # the engines' per-step poll (no device sync)
            p2p.poll()
    dist.barrier()
    p2p.destroy()


@pytest.mark.parametrize("protocol", ["ll", "flag"])
def test_p2p_allreduce_two_processes_one_gpu(protocol):
    run_gloo(_worker, 2, protocol)


@pytest.mark.parametrize("protocol", ["ll", "flag"])
def test_p2p_allreduce_four_processes_one_gpu(protocol):
    run_gloo(_worker, 4, protocol)


@pytest.mark.parametrize("protocol", ["ll", "flag"])
def test_p2p_allreduce_timeout_flags_error(protocol):
    run_gloo(_timeout_worker, 2, protocol)


def test_rccl_watchdog_aborts_stalled_collective():
    """Verdict r2 item 3: a collective that never completes ends in ncclCommAbort + a RuntimeError
    on the training thread within DTA_COMM_TIMEOUT_S, instead of a hang.  RCCL refuses two ranks on
    one GPU, so the stall is an injected never-completing event on a real one-rank RcclComm; the
    abort is the real ncclCommAbort (later collectives on the aborted communicator raise too)."""
    import time

    from distributed_training_amd.parallel.comm import RcclComm

    dev = torch.device("cuda", 0)
    comm = RcclComm(0, 1, dev, timeout_s=1.0)
    x = torch.ones(1024, device=dev)
    comm.all_reduce(x)  # a real one: completes, tracked and retired
    torch.cuda.synchronize()

    class Stalled:
        def query(self):
            return False

    comm.watchdog.exit_grace_s = 60.0
    t0 = time.monotonic()
    comm.watchdog.track(Stalled(), "injected stalled all_reduce")
    with pytest.raises(RuntimeError, match="injected stalled all_reduce"):
        while time.monotonic() - t0 < 10.0:
            comm.poll_errors()
            time.sleep(0.05)
    assert time.monotonic() - t0 < 5.0
    assert comm.aborted
    with pytest.raises(RuntimeError):
        comm.all_reduce(x)
