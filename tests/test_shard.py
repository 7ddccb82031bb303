"""Multi-rank path on CPU: frame sharding + the bench's collectives over gloo (world_size 2)."""
import os
import socket

import pytest

from zwebp.shard import frame_seed, gather_counts, rank_frames, reduce_max, shard_range


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (7, 2), (512, 8), (4096, 8), (5, 3)])
def test_shard_range_partitions(n, world):
    seen = []
    for r in range(world):
        s, e = shard_range(n, r, world)
        assert 0 <= s <= e <= n
        seen += list(range(s, e))
    assert seen == list(range(n))
    sizes = [shard_range(n, r, world)[1] - shard_range(n, r, world)[0] for r in range(world)]
    assert max(sizes) - min(sizes) <= 1


def test_frame_seed():
    assert frame_seed(0) == 0x5EED0000 and frame_seed(3) == 0x5EED0003


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s, e = shard_range(10, rank, world)
    el = reduce_max(0.5 + rank)
    counts = gather_counts([rank, e - s])
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, s, e, el, counts))


def test_gloo_world2_collectives():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(r[1], r[2]) for r in res] == [(0, 5), (5, 10)]
    assert all(r[3] == 1.5 for r in res)
    assert res[0][4] == [[0, 5], [1, 5]]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_rank_frames_config5_split(world):
    """BASELINE config 5: 4096 frames split over N ranks cover every frame once."""
    got = []
    for r in range(world):
        s, n = rank_frames(r, world, 0, 4096)
        got += list(range(s, s + n))
    assert sorted(got) == list(range(4096))
    assert rank_frames(1, 2, 1024, 0) == (1024, 1024)  # weak scaling: every rank its own F frames


def _bench_split_worker(rank, world, port, q):
    """The bench's frame assignment and its collectives over gloo: per-rank
    frame counts all-gathered, max time all-reduced, verification counts summed."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = rank_frames(rank, world, 1024, 4096)
    steps = 3
    total = sum(c[0] for c in gather_counts([n * steps]))
    el = reduce_max(1.0 + 0.25 * rank)
    seeds = [frame_seed(first + i) for i in range(4)]
    vc = gather_counts([n, 0, 0])
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, first, n, total, el, seeds, [sum(c[i] for c in vc) for i in range(3)]))


def test_gloo_world2_config5_split():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_split_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(r[1], r[2]) for r in res] == [(0, 2048), (2048, 2048)]
    assert all(r[3] == 4096 * 3 for r in res)          # value numerator: frames of all ranks
    assert all(r[4] == 1.25 for r in res)              # max over ranks
    assert res[1][5][0] == frame_seed(2048)            # rank 1's distinct frames start at its block
    assert all(r[6] == [4096, 0, 0] for r in res)      # verification counts summed over ranks
