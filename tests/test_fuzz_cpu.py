"""Property tests (hypothesis) for the T0 tier of SURVEY §4.2: sharding arithmetic (R5, every
remainder policy), the C++ min-max partitioner against brute force, the bucket planner, and the
pipeline compute orders (every schedule runs each (chunk, microbatch) forward exactly once before
its backward)."""
import itertools

from hypothesis import given, settings, strategies as st

from madnn.data import shard, shard_bounds
from madnn.ops import native_runtime as nr


@settings(max_examples=60, deadline=None)
@given(n=st.integers(0, 500), world=st.integers(1, 9))
def test_shard_bounds_drop_and_last(n, world):
    spans = [shard_bounds(n, r, world, "drop") for r in range(world)]
    # drop: equal disjoint contiguous stripes, remainder dropped (reference datamodule.lua:239-246)
    assert all(e - s == n // world for s, e in spans)
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    last = [shard_bounds(n, r, world, "last") for r in range(world)]
    covered = sorted(i for s, e in last for i in range(s, e))
    assert covered == list(range(n))  # last: the final rank takes the remainder


@settings(max_examples=40, deadline=None)
@given(n=st.integers(1, 200), world=st.integers(1, 8))
def test_shard_pad_and_strided(n, world):
    data = list(range(n))
    pads = [shard(data, r, world, "pad") for r in range(world)]
    assert len({len(p) for p in pads}) == 1  # every rank the same count
    assert set(itertools.chain(*pads)) == set(data)  # nothing dropped
    strided = [shard(data, r, world, strided=True) for r in range(world)]
    flat = sorted(itertools.chain(*strided))
    assert flat == sorted(set(flat)) and len(flat) == (n // world) * world


def _brute(costs, k):
    best = float("inf")
    L = len(costs)
    for cuts in itertools.combinations(range(1, L), k - 1):
        b = [0, *cuts, L]
        best = min(best, max(sum(costs[b[i]:b[i + 1]]) for i in range(k)))
    return best


@settings(max_examples=40, deadline=None)
@given(costs=st.lists(st.floats(0.1, 10.0), min_size=2, max_size=9), k=st.integers(1, 4))
def test_partition_matches_brute_force(costs, k):
    k = min(k, len(costs))
    bounds, best = nr.partition(costs, k)
    assert bounds[0] == 0 and bounds[-1] == len(costs) and len(bounds) == k + 1
    assert all(bounds[i] < bounds[i + 1] for i in range(k))
    got = max(sum(costs[bounds[i]:bounds[i + 1]]) for i in range(k))
    assert abs(got - best) < 1e-6 * max(1.0, best)
    assert abs(best - _brute(costs, k)) < 1e-6 * max(1.0, best)


@settings(max_examples=40, deadline=None)
@given(numels=st.lists(st.integers(0, 5000), min_size=1, max_size=30), cap=st.integers(1, 20000))
def test_bucket_plan_is_a_packing(numels, cap):
    bucket_of, offset_of, sizes = nr.plan_buckets(numels, cap, 16)
    for i, n in enumerate(numels):
        b = bucket_of[i]
        assert 0 <= b < len(sizes)
        assert offset_of[i] % 16 == 0 and offset_of[i] + n <= sizes[b]
    for b in range(len(sizes)):  # no two tensors of a bucket overlap
        spans = sorted((offset_of[i], offset_of[i] + numels[i]) for i in range(len(numels)) if bucket_of[i] == b)
        assert all(spans[j][1] <= spans[j + 1][0] for j in range(len(spans) - 1))


@settings(max_examples=40, deadline=None)
@given(kind=st.sampled_from(["gpipe", "1f1b", "interleaved"]), stages=st.integers(1, 4), mult=st.integers(1, 4),
       chunks=st.integers(1, 3))
def test_pipeline_orders_are_complete(kind, stages, mult, chunks):
    nmicro = stages * mult
    v = chunks if kind == "interleaved" else 1
    for s in range(stages):
        order = nr.pipeline_order(kind, s, stages, nmicro, v)
        fwd = [(c, m) for op, c, m in order if op == "F"]
        bwd = [(c, m) for op, c, m in order if op == "B"]
        want = sorted((c, m) for c in range(v) for m in range(nmicro))
        assert sorted(fwd) == want and sorted(bwd) == want
        pos = {("F", c, m): i for i, (op, c, m) in enumerate(order) if op == "F"}
        assert all(pos[("F", c, m)] < i for i, (op, c, m) in enumerate(order) if op == "B")
