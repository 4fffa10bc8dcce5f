"""Debug: compressor fix-up variants vs the oracle (diff positions, determinism)."""
import sys, os
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for p in (R, os.path.join(R, "oracle"), os.path.join(R, "audio-mastering-engine_amd"), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import numpy as np
import oracle
from amx import synth
from test_gpu_parity import C3, _chunk_chain

fs = 48000
n = int(fs * 9.7)
for sig in ["mix", "music"]:
    x = synth.mix_like(n, fs, 2, seed=7) if sig == "mix" else synth.music_like(n, fs, 2, seed=7, peak_dbfs=-3.0)
    x16 = oracle.quantize(x)
    chunks = [(0, n // 2 + 3), (n // 2 + 3, n - (n // 2 + 3))]
    ref = np.concatenate([oracle.chunk(x16[s:s + m], fs, C3) for s, m in chunks])
    for warm, rounds in [(0, 0), (0, 1), (0, 1), (0, 2), (0, 3), (64, 1), (2048, 1), (2048, 2)]:
        out, _ = _chunk_chain(x16, fs, dict(C3, _env_warm=warm, _env_rounds=rounds), chunks)
        d = np.abs(out.astype(np.int32) - ref.astype(np.int32)).max(axis=1)
        bad = np.nonzero(d)[0]
        print(sig, warm, rounds, "max", d.max(), "nbad", bad.size,
              "first", bad[:3].tolist(), "last", bad[-3:].tolist(), flush=True)
