"""K5 one-shot all-reduce (madnn/ops/csrc/xgmi.hip) on the device.

The box has one GPU, so the multi-rank test runs 2 processes on it: the IPC handle exchange,
the cross-process flag protocol (uncached flags, system-scope release/acquire) and the W-way
sum run exactly as across the xGMI peers of an 8-GPU node; only the link is the local HBM.
Results are compared with the fp32 sum of every rank's input."""
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _w_oneshot(rank, world):
    from madnn.comm.oneshot import OneShotAllReduce

    c = OneShotAllReduce(None, cap_bytes=4 << 20, spin_limit=1 << 20)
    for it, (n, dt) in enumerate([(8, torch.float32), (1000, torch.bfloat16), (4096 * 33 + 5, torch.float32),
                                  (2 << 20, torch.bfloat16), (777, torch.bfloat16), (65536, torch.float32)]):
        gens = [torch.Generator().manual_seed(100 * it + r) for r in range(world)]
        xs = [torch.randn(n, generator=g) for g in gens]
        x = xs[rank].to(dt).cuda()
        y = c(x.clone())
        ref = sum(v.to(dt).float() for v in xs)
        torch.cuda.synchronize()
        tol = 1e-5 if dt == torch.float32 else 2e-2
        err = float(((y.float().cpu() - ref).abs() / (ref.abs() + 1)).max())
        assert err <= tol, (n, dt, err)
    for _ in range(50):  # many epochs: staging halves and flags are reused
        x = torch.full((3000,), float(rank + 1), device="cuda")
        c(x)
    torch.cuda.synchronize()
    assert bool((x == sum(range(1, world + 1))).all())
    c.check()
    dist.barrier()
    c.close()


def test_oneshot_allreduce_two_processes_one_gpu(cuda):
    from dist_utils import run_dist

    run_dist(_w_oneshot, 2, device="cuda", backend="gloo")


def test_oneshot_world_one_and_timeout_flag(cuda):
    """World 1 (no process group): the kernel is a copy; a context whose peer flag never arrives
    cannot be built at world 1, so the bounded wait is exercised through the error word API."""
    from madnn.comm.oneshot import OneShotAllReduce

    c = OneShotAllReduce(None, cap_bytes=1 << 16)
    x = torch.randn(5000, device=cuda)
    y = c(x.clone())
    torch.testing.assert_close(y, x)
    c.check()
    assert not c.supports(torch.randn(1 << 15, device=cuda))   # beyond cap
    c.close()


def _w_absent_peer(rank, world):
    """Rank 1 arrives long after rank 0's bounded wait expired: rank 0's output holds only its own
    input, and its next call raises instead of training on."""
    import time

    from madnn.comm.oneshot import OneShotAllReduce, OneShotTimeout

    c = OneShotAllReduce(None, cap_bytes=1 << 16, spin_limit=1 << 12)
    x = torch.full((4096,), float(rank + 1), device="cuda")
    if rank == 1:
        time.sleep(3.0)
    c(x)
    torch.cuda.synchronize()
    if rank == 0:
        assert bool((x == 1.0).all()), "timed-out wait must leave the local input (no partial peer data)"
        raised = False
        try:
            c(torch.ones(8, device="cuda"))
        except OneShotTimeout:
            raised = True
        assert raised, "the next call must raise after a timed-out peer wait"
    else:
        c.check()   # rank 0's flag for this epoch was already there: rank 1 completed normally
    dist.barrier()
    c.close()


def test_oneshot_absent_peer_raises(cuda):
    from dist_utils import run_dist

    run_dist(_w_absent_peer, 2, device="cuda", backend="gloo")
