"""N > 1 path on the CPU: the chunk-sharded exchange steps of amx/dist.py run over
gloo with world_size 2 (the same functions run over RCCL on the GPU path).

The device kernels are replaced by a float64 numpy restatement of the K-weighting
filter (libebur128's direct-form II, the oracle's coefficients), so what is checked
here is the sharding algebra and the collective plumbing: zero-start tails ->
all-gather -> carry composition (dist.carry_from_tails) reproduces the state the
sequential filter has at each rank boundary, the all-reduced hop energies and peaks
equal the single-process ones, the limiter halo arrives from the previous rank and
the sequential limiter state is handed along in rank order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from amx import dist as adist
from amx.chunking import chunk_bounds

FS = 48000
HOP = 4800


def _coefs():
    import oracle
    return oracle.kweight_coefs(FS)


def _kfilter(x, state, b, a):
    """libebur128 DF-II over x [n, 2] float64 from state [2, 4]; returns (y, state)."""
    v = np.array(state, np.float64).copy()
    y = np.empty_like(x)
    for i in range(x.shape[0]):
        v0 = x[i] - a[1] * v[:, 0] - a[2] * v[:, 1] - a[3] * v[:, 2] - a[4] * v[:, 3]
        y[i] = b[0] * v0 + b[1] * v[:, 0] + b[2] * v[:, 1] + b[3] * v[:, 2] + b[4] * v[:, 3]
        v[:, 3] = v[:, 2]
        v[:, 2] = v[:, 1]
        v[:, 1] = v[:, 0]
        v[:, 0] = v0
    return y, v


def _propagator(a):
    A = np.zeros((4, 4))
    A[0, :] = -np.asarray(a[1:5])
    A[1, 0] = A[2, 1] = A[3, 2] = 1.0

    def propagate(frames, s8):
        P = np.linalg.matrix_power(A, int(frames))
        s = np.asarray(s8, np.float64).reshape(2, 4)
        return (s @ P.T).reshape(8)
    return propagate


def _hops(y, t0, n_hops):
    """energy per 100 ms hop of the whole-track timeline for frames [t0, t0 + len(y))."""
    h = np.zeros((n_hops, 2))
    t = t0 + np.arange(y.shape[0])
    np.add.at(h, t // HOP, y * y)
    return h


def _signal(n, seed=5):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / FS
    x = 0.3 * np.sin(2 * np.pi * 220 * t)[:, None] + 0.05 * rng.standard_normal((n, 2))
    x[n // 3:n // 3 + 700] *= 3.0
    return x


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, spans):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b, a = _coefs()
        n = sum(spans)
        x = _signal(n)
        t0 = sum(spans[:rank])
        mine = x[t0:t0 + spans[rank]]
        n_hops = n // HOP + 1

        # 1. zero-start tail -> all-gather -> carry
        _, tail = _kfilter(mine, np.zeros((2, 4)), b, a)
        tails_all = torch.zeros((world, 2, 4), dtype=torch.float64)
        adist.gather_tails(torch.from_numpy(tail), tails_all)
        carry = adist.carry_from_tails(tails_all.numpy().reshape(world, 8), spans, rank, _propagator(a))
        _, s_true = _kfilter(x[:t0], np.zeros((2, 4)), b, a)
        np.testing.assert_allclose(carry.reshape(2, 4), s_true, rtol=1e-10, atol=1e-13)

        # 2. hop partials from the carried state, all-reduced
        y, _ = _kfilter(mine, carry.reshape(2, 4), b, a)
        hops = torch.from_numpy(_hops(y, t0, n_hops))
        peak = torch.from_numpy(np.abs(mine).max(axis=0))
        adist.reduce_loudness(hops, peak)
        y_all, _ = _kfilter(x, np.zeros((2, 4)), b, a)
        np.testing.assert_allclose(hops.numpy(), _hops(y_all, 0, n_hops), rtol=1e-10, atol=1e-12)
        np.testing.assert_array_equal(peak.numpy(), np.abs(x).max(axis=0))
        # loudnorm off: peaks only
        pk = torch.full((2,), float(rank))
        adist.reduce_loudness(None, pk)
        assert pk.tolist() == [world - 1.0] * 2

        # 3. limiter halo: the previous rank's last h frames (zero-padded when short)
        out16 = torch.from_numpy((mine * 8000).astype(np.int16))
        for h in (37, spans[0] + 5):
            prev = adist.gather_halo(out16, spans[rank], h, rank, world)
            if rank == 0:
                assert prev is None
            else:
                p_out = (x[:spans[0]] * 8000).astype(np.int16)
                want = p_out[max(0, spans[0] - h):]
                want = np.concatenate([np.zeros((h - want.shape[0], 2), np.int16), want])
                np.testing.assert_array_equal(prev.numpy(), want)

        # 4. sequential limiter state, rank to rank
        st = torch.zeros(3, dtype=torch.float64)
        order = []

        def run():
            order.append(st.tolist())
            st.mul_(10.0).add_(rank + 1)
        adist.chain_state(st, run, rank, world)
        assert order[0] == ([0.0] * 3 if rank == 0 else [float(sum((q + 1) * 10 ** (rank - 1 - q) for q in range(rank)))] * 3)

        # 5. speculative hand-off: every rank runs from rest first; a rank re-runs only
        # when the state it receives is not the rest state.  Toy limiter on the real
        # state layout (B = 4): rank 0 ends at rest when `rest0`, else with att = 0.5;
        # ranks > 0 end at rest.
        bs = 4
        for rest0 in (True, False):
            sv = torch.zeros(8 + 3 * bs, dtype=torch.float64)
            seen = []

            def lim_run():
                seen.append(float(sv[0]))
                sv.zero_()
                sv[5] = 1.0
                sv[8 + 2 * bs:] = -1.0
                sv[0] = 1.0 if (rank > 0 or rest0) else 0.5
            adist.chain_state_speculative(sv, lim_run, lambda v: adist.is_rest_state(v, bs), rank, world)
            if rank == 0:
                assert seen == [0.0]                      # one run, from nothing carried
            else:
                assert seen == ([0.0] if rest0 else [0.0, 0.5])   # re-run from the received state
            assert adist.is_rest_state(sv, bs) == (rank > 0 or rest0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("spans", [(9000, 13500), (4700, 4900)])
def test_sharded_exchanges_gloo_world2(spans):
    """world_size 2 over gloo: spans not multiples of the hop, so one hop straddles
    the boundary and gets one addend from each rank."""
    mp.spawn(_worker, args=(2, _free_port(), list(spans)), nprocs=2, join=True)


def test_carry_three_spans():
    """carry_from_tails over three ranks' spans equals the sequential filter state."""
    b, a = _coefs()
    spans = [3001, 4800, 2500]
    x = _signal(sum(spans), seed=9)
    tails, t0 = [], 0
    for n in spans:
        tails.append(_kfilter(x[t0:t0 + n], np.zeros((2, 4)), b, a)[1].reshape(8))
        t0 += n
    for r in range(3):
        c = adist.carry_from_tails(tails, spans, r, _propagator(a))
        s = _kfilter(x[:sum(spans[:r])], np.zeros((2, 4)), b, a)[1]
        np.testing.assert_allclose(c.reshape(2, 4), s, rtol=1e-10, atol=1e-13)


@pytest.mark.parametrize("n_chunks,world", [(1, 1), (10, 1), (10, 2), (10, 3), (64, 8), (9, 8)])
def test_shard_ranges(n_chunks, world):
    r = adist.shard_ranges(n_chunks, world)
    assert len(r) == world and r[0][0] == 0 and r[-1][1] == n_chunks
    assert all(r[i][1] == r[i + 1][0] for i in range(world - 1))
    sizes = [b - a for a, b in r]
    assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


@pytest.mark.parametrize("frames,world", [
    ([11520000] * 64, 8), ([5, 1, 1, 1, 1, 5], 3), ([3, 3], 2), ([1] * 9, 8), ([100, 1, 1, 1], 2)])
def test_shard_tracks(frames, world):
    """C4 batches: contiguous whole-track runs, every rank non-empty, balanced."""
    r = adist.shard_tracks(frames, world)
    assert len(r) == world and r[0][0] == 0 and r[-1][1] == len(frames)
    assert all(r[i][1] == r[i + 1][0] for i in range(world - 1))
    assert all(b > a for a, b in r)
    if len(set(frames)) == 1 and len(frames) % world == 0:
        assert all(b - a == len(frames) // world for a, b in r)


def test_shard_geometry_matches_one_gpu_timeline():
    """Rank spans tile the single-GPU output timeline: the per-chunk output lengths
    (pydub overlay rounding when multiband) summed per rank, in order."""
    fs = 48000
    frames = fs * 95 + 123
    bounds = chunk_bounds(frames, fs, 512)
    for mb in (False, True):
        out_n = [adist.chunk_out_frames(n, fs, mb) for _, n in bounds]
        for world in (1, 2, 3):
            ranges = adist.shard_ranges(len(bounds), world)
            span = [sum(out_n[a:b]) for a, b in ranges]
            assert sum(span) == sum(out_n)
            t0 = [sum(out_n[:a]) for a, _ in ranges]
            assert t0 == [sum(span[:r]) for r in range(world)]
        if not mb:
            assert out_n == [n for _, n in bounds]


def _batch_worker(rank, world, port, frames):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = adist.shard_tracks(frames, world)
        mine = torch.tensor(list(r[rank]), dtype=torch.int64)
        allr = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, mine)
        got = [tuple(int(v) for v in t) for t in allr]
        # every rank derives the same split on its own: the runs tile the batch in
        # order, no rank is empty, no track is in two ranks (no exchange needed)
        assert got == r
        assert got[0][0] == 0 and got[-1][1] == len(frames)
        assert all(got[i][1] == got[i + 1][0] for i in range(world - 1))
        assert all(b > a for a, b in got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("frames", [[11520000] * 16, [5, 1, 1, 1, 1, 5, 2]])
def test_batch_split_gloo_world2(frames):
    """C4 batch split over two ranks (gloo): each rank's ShardedBatch share, agreed
    without any exchange of data."""
    mp.spawn(_batch_worker, args=(2, _free_port(), frames), nprocs=2, join=True)


def test_sharded_track_mode_word():
    """A chunk-sharded step reads k_decide's control word (bit 0 limiter idle, bits 4..7
    loudnorm mode): mode 3 sends the track to loudnorm's dynamic path
    (ShardedTrack.dynamic) instead of the linear finalisation."""
    for mode in (0, 1, 2):
        for fast in (0, 1):
            assert not adist.is_dynamic((mode << 4) | fast)
    for fast in (0, 1):
        assert adist.is_dynamic((3 << 4) | fast)


def _gather_worker(rank, world, port, spans):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        whole = torch.arange(2 * sum(spans), dtype=torch.int32).to(torch.int16).reshape(-1, 2)
        f0 = sum(spans[:rank])
        out = torch.zeros((spans[rank] + 7, 2), dtype=torch.int16)    # a span buffer with a tail
        out[:spans[rank]] = whole[f0:f0 + spans[rank]]
        got = adist.gather_track(out, spans[rank], spans, world)
        assert torch.equal(got, whole)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("spans", [[5, 3], [1, 9], [4, 4]])
def test_gather_track_gloo_world2(spans):
    """dynamic mode's span gather (ShardedTrack.dynamic): spans of different lengths are
    padded to the longest for one all_gather_into_tensor and reassembled in rank order"""
    mp.spawn(_gather_worker, args=(2, _free_port(), spans), nprocs=2, join=True)


@pytest.mark.parametrize("K,k_fin,world", [(188, 181, 2), (188, 181, 8), (9, 2, 2), (12, 5, 4), (40, 33, 3)])
def test_shard_segments(K, k_fin, world):
    """the sharded dynamic mode's segment split: contiguous runs tiling [0, K), every rank
    non-empty, no boundary inside the FINAL flush frame's segments [k_fin, K)"""
    r = adist.shard_segments(K, k_fin, world)
    assert len(r) == world and r[0][0] == 0 and r[-1][1] == K
    assert all(r[i][1] == r[i + 1][0] for i in range(world - 1))
    assert all(b > a for a, b in r)
    assert all(b <= k_fin for a, b in r[:-1]) and r[-1][0] < k_fin
    pre = [min(b, k_fin) - a for a, b in r]
    assert max(pre) - min(pre) <= 1


def test_shard_segments_short_track():
    """fewer pre-FINAL segments than ranks: no split (every rank runs the filter whole)"""
    assert adist.shard_segments(30, 1, 2) is None
    assert adist.shard_segments(35, 7, 8) is None
    assert adist.shard_segments(36, 8, 8) is not None
