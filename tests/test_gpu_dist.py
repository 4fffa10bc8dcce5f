"""N = 2 rehearsal of the chunk-sharded path on one GPU: two processes, both on
cuda:0, exchanging over gloo (host-staged) instead of RCCL.  Every device kernel of
the N > 1 path runs -- K-filter tails and carry, hop partials, all-reduced loudness,
the limiter halo and, when the limiter can engage, the rank-to-rank sequential
limiter -- and the concatenated rank outputs must equal the one-rank run of the
same track bit for bit (the chunking, loudness decision and limiter are all
track-level, so sharding must not change a sample), and the C oracle's whole
pipeline on the same input."""
import datetime
import gc
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FS = 48000
MB = dict(multiband=True, low_thresh=-25.0, low_ratio=6.0, mid_thresh=-20.0, mid_ratio=3.0,
          high_thresh=-15.0, high_ratio=4.0)
CASES = {
    "c3_lufs": dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0,
                    lufs=-14.0, width=1.3, analog_character=40.0, **MB),
    "loud_limiter": dict(width=1.5),       # no EQ stage (the EQ lowers the level): clips
    # a full-scale square: the limiter never comes to rest, so rank 1's first run (from
    # rest) is wrong and it must re-run from the state rank 0 hands it
    "square_limiter": dict(),
    # 44.1 kHz: rank 1's span starts off the 192 kHz phase grid (147 chain frames per 640
    # outputs), so its resampler segments run with a non-zero phase pattern (k_up_poly)
    "c3_lufs_44k1": dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0,
                         lufs=-14.0, width=1.3, analog_character=40.0, **MB),
    # quiet programme with sparse full-scale transients: TP + offset > -1.5 dBTP, so
    # loudnorm's pass 2 takes dynamic mode and the output is the 192 kHz stream
    "dynamic": dict(bass_boost=1.0, lufs=-14.0),
    # the same with one-frame filter segments and no warm-up (AMX_LN_SEG=1, AMX_LN_WARM=0):
    # most segments start from a wrong guess, so the limiter state rank 0's walk hands
    # rank 1 decides rank 1's first segment
    "dynamic_nowarm": dict(bass_boost=1.0, lufs=-14.0),
    # 44.1 kHz: the ranks' 192 kHz ranges of the filter come from the generic (M > 1)
    # resampler form, each rank upsampling only what its segments read
    "dynamic_44k1": dict(bass_boost=1.0, lufs=-14.0),
    # a quiet 6 s intro: the filter starts below measured_thresh (above_threshold 0), a
    # feedback loop: rank 0 runs those frames in order up to the hand-over segment and
    # broadcasts the control words and deltas, then every rank runs its own windows
    "dynamic_quiet": dict(bass_boost=1.0, lufs=-14.0),
    # quiet past rank 0's segments (62 s of 75): the split hand-over cannot run there
    "dynamic_quiet_long": dict(bass_boost=1.0, lufs=-14.0),
}
ENV = {"dynamic_nowarm": {"AMX_LN_SEG": "1", "AMX_LN_WARM": "0"}}
RATE = {"c3_lufs_44k1": 44100, "dynamic_44k1": 44100}


# input gain per case: the loud case drives 0.1 % of the frames over the limit, so the final
# alimiter (limit 0.98) must engage and the ranks hand its state along
GAIN = {"c3_lufs": 1.0, "loud_limiter": 1.3, "square_limiter": 1.0, "c3_lufs_44k1": 1.0, "dynamic": 1.0,
        "dynamic_nowarm": 1.0, "dynamic_44k1": 1.0, "dynamic_quiet": 1.0, "dynamic_quiet_long": 1.0}


def _track(seconds, case):
    from amx import synth
    fs = RATE.get(case, FS)
    n = int(fs * seconds)
    if case == "square_limiter":
        return synth.square(n, fs, 2, freq=110.0, amp=1.0)
    if case.startswith("dynamic"):
        x = synth.mix_like(n, fs, 2, seed=11) * 0.12
        rng = np.random.default_rng(11)
        for k in rng.integers(0, n - 200, max(2, int(seconds * 2))):
            x[k:k + 50] += rng.uniform(-0.9, 0.9, (50, 2))
        if case == "dynamic_quiet":
            x[:int(6 * fs)] *= 0.0005
        if case == "dynamic_quiet_long":
            x[:int(62 * fs)] *= 0.0005
        return np.clip(x, -1.0, 1.0).astype(np.float32)
    return (synth.mix_like(n, fs, 2, seed=3) * np.float32(GAIN[case])).astype(np.float32)


def _worker(rank, world, port, case, seconds, outdir):
    import torch
    import torch.distributed as dist
    from amx.dist import ShardedTrack
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.update(ENV.get(case, {}))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    try:
        torch.cuda.set_device(0)
        x = _track(seconds, case)
        tr = ShardedTrack(RATE.get(case, FS), 2, CASES[case], x.shape[0], rank, world, quantum=512)
        d_in = torch.from_numpy(np.ascontiguousarray(x[tr.in0:tr.in0 + tr.local_frames])).cuda()
        y = tr.step(d_in)
        torch.cuda.synchronize()
        y_eager = y.cpu().numpy()
        # the same step from captured graph segments (bench.py's timed path)
        tr.capture(d_in)
        y_graph = tr.replay().cpu().numpy()
        np.testing.assert_array_equal(y_graph, y_eager)
        np.save(os.path.join(outdir, "y%d.npy" % rank), y_eager)
        fast = bool(int(tr.job.ctl[0].item()) & 1)
        np.save(os.path.join(outdir, "fast%d.npy" % rank), np.array([fast]))
        if case.startswith("dynamic"):
            with open(os.path.join(outdir, "form%d.txt" % rank), "w") as f:
                f.write(tr.dyn_info["form"])
        elif not fast:
            # the in-graph limiter runs from rest (amx_final_desc.from_rest)
            # while the state buffer holds the previous step's valid end state; a changed
            # input must still give the eager step's output, hand-off included
            d_in.neg_()
            y_graph2 = tr.replay().cpu().numpy()
            y_eager2 = tr.step(d_in).cpu().numpy()
            np.testing.assert_array_equal(y_graph2, y_eager2)
            assert not np.array_equal(y_graph2, y_graph)
        tr.close()
    finally:
        dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("case", sorted(CASES))
def test_two_ranks_match_one(gpu, case):
    import torch
    import torch.multiprocessing as mp
    from amx.dist import ShardedTrack
    # 3 chunks -> ranks own 2 + 1; the sequential-limiter case 2 chunks (that path walks
    # every frame in order)
    seconds = 75.0 if case.startswith("c3_lufs") or case.startswith("dynamic") else 32.0
    x = _track(seconds, case)
    if case.startswith("dynamic"):
        # the reference: the oracle's whole pipeline in dynamic mode (the ranks' filter
        # gains come from the step's own all-reduced hop energies, which equal the
        # one-GPU sums up to rounding beside a rank boundary: within 3 LSB)
        import oracle
        from amx.chunking import chunk_bounds
        fs = RATE.get(case, FS)
        y1, rinfo = oracle.pipeline(oracle.quantize(x), fs, CASES[case], chunk_bounds(x.shape[0], fs, 512))
        assert rinfo["mode"] == "dynamic" and rinfo["sample_rate"] == 192000
    else:
        one = ShardedTrack(RATE.get(case, FS), 2, CASES[case], x.shape[0], 0, 1, quantum=512)
        y1 = one.step(torch.from_numpy(np.ascontiguousarray(x)).cuda()).cpu().numpy()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _port(), case, seconds, d), nprocs=2, join=True)
        parts = [np.load(os.path.join(d, "y%d.npy" % r)) for r in range(2)]
        fast = [bool(np.load(os.path.join(d, "fast%d.npy" % r))[0]) for r in range(2)]
        forms = [open(os.path.join(d, "form%d.txt" % r)).read() if case.startswith("dynamic") else None
                 for r in range(2)]
    y2 = np.concatenate(parts)
    assert fast[0] == fast[1]
    if case.startswith("dynamic"):
        # both filter runs on the ranks' windows, with the limiter-state hand-off (a quiet
        # start: the whole filter on every rank)
        # a quiet start runs split (rank 0 in order up to the hand-over);
        # one still quiet past rank 0's segments takes the replicated form
        want = "replicated" if case == "dynamic_quiet_long" else "windowed"
        assert forms == [want] * 2, forms
    # the loud case must exercise the rank-to-rank sequential limiter
    if not case.startswith("dynamic"):
        assert fast[0] == case.startswith("c3_lufs"), "limiter fast path %s" % fast[0]
    assert y2.shape == y1.shape
    diff = np.abs(y2.astype(np.int32) - y1.astype(np.int32))
    if case.startswith("dynamic"):
        exact = float((diff == 0).mean())
        print("%s over 2 ranks vs the oracle: max |diff| %d LSB, exact %.7f" % (case, diff.max(), exact))
        assert diff.max() <= 3 and exact >= 0.999, (int(diff.max()), exact)
        return
    assert diff.max() == 0, "max |diff| %d LSB at %s (limiter fast path %s)" % (
        diff.max(), np.argmax(diff.max(axis=1)), fast[0])
    # and against the oracle's whole pipeline (the N = 2 linear cases were
    # checked against the one-rank GPU run only); the same bound as the one-GPU
    # pipeline tests (tests/test_gpu_parity.py)
    import oracle
    from amx.chunking import chunk_bounds
    fs = RATE.get(case, FS)
    yo, oinfo = oracle.pipeline(oracle.quantize(x), fs, CASES[case], chunk_bounds(x.shape[0], fs, 512))
    assert yo.shape == y2.shape, (yo.shape, y2.shape)
    do = np.abs(y2.astype(np.int32) - yo.astype(np.int32))
    exact = float((do == 0).mean())
    print("%s over 2 ranks vs the oracle: max |diff| %d LSB, exact %.7f" % (case, do.max(), exact))
    assert do.max() <= 3 and exact >= 0.9999, (int(do.max()), exact)


@pytest.mark.parametrize("case", ["c3_lufs", "square_limiter"])
def test_rccl_forced_exchange_world1(gpu, case):
    """RCCL rehearsal on one GPU (RCCL refuses two ranks on one device): a one-rank
    "nccl" process group with ShardedTrack's exchanges forced on, so the N > 1 step --
    one captured graph, the edge and tail/peak all_gather_into_tensor, the hop all_reduce,
    the device carry kernels, the limiter on the device's decision -- runs through RCCL.
    Eager step and graph replay must equal the bypass path bit for bit."""
    import torch
    import torch.distributed as dist
    from amx.dist import ShardedTrack
    seconds = 75.0 if case == "c3_lufs" else 32.0
    x = _track(seconds, case)
    d_in = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    ref = ShardedTrack(FS, 2, CASES[case], x.shape[0], 0, 1, quantum=512)
    y_ref = ref.step(d_in).cpu().numpy()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=60))
    tr = None
    try:
        assert dist.get_backend() == "nccl"
        tr = ShardedTrack(FS, 2, CASES[case], x.shape[0], 0, 1, quantum=512, force_exchange=True)
        y_eager = tr.step(d_in).cpu().numpy()
        tr.capture(d_in)
        # the N > 1 step as ONE graph per slot: the RCCL collectives are captured nodes;
        # the two slots alternate, a step resolved when the next one is enqueued
        assert isinstance(tr._g, list) and len(tr._g) == 1 and len(tr._slots) == 2
        tr.replay()
        y_graph = tr.flush().cpu().numpy()
        for _ in range(3):
            tr.replay()
        y_graph2 = tr.flush().cpu().numpy()
        torch.cuda.synchronize()
        # each slot's in-graph limiter run writes its end state into
        # that slot's own lim_state (what _resolve hands to the next rank), and a changed
        # input between replays gives the eager output
        lim_slots = [sl["job"].lim_state.clone() for sl in tr._slots]
        d_in.neg_()
        tr.replay()
        tr.replay()
        y_graph3 = tr.flush().cpu().numpy()
        ref2 = ShardedTrack(FS, 2, CASES[case], x.shape[0], 0, 1, quantum=512)
        y_ref3 = ref2.step(d_in).cpu().numpy()
        lim_ref3 = ref2.job.lim_state.clone()
        lim_slots3 = [sl["job"].lim_state.clone() for sl in tr._slots]
        ref2.close()
    finally:
        # the slots' graphs hold RCCL nodes of this group's communicator: free them (and
        # everything they reference) before the group, not at some later collection
        if tr is not None:
            tr.close()
        tr = None
        gc.collect()
        torch.cuda.synchronize()
        dist.destroy_process_group()
    ref.close()
    np.testing.assert_array_equal(y_eager, y_ref)
    np.testing.assert_array_equal(y_graph, y_ref)
    np.testing.assert_array_equal(y_graph2, y_ref)
    np.testing.assert_array_equal(y_graph3, y_ref3)
    assert not np.array_equal(y_graph3, y_graph)
    if case == "square_limiter":            # the general limiter engaged: its end state
        for k in range(2):
            assert float(lim_slots[k][0, 5]) == 1.0          # written (valid) by the graph
            np.testing.assert_array_equal(lim_slots3[k].cpu().numpy(), lim_ref3.cpu().numpy())
