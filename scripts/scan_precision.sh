#!/bin/bash
# The two-pass IIR's precision on the CPU: one 30 s 96 kHz channel of
# the C3 EQ through scripts/scan_precision_emu.cpp with the scan tables / accumulation in
# double or long double, against the sequential double and 80-bit recursions.
set -e
cd "$(dirname "$0")/.."
W=$(mktemp -d)
python3 - "$W" <<'PY'
import sys
sys.path[:0] = ['audio-mastering-engine_amd', 'oracle']
import numpy as np, oracle
from amx import synth
w = sys.argv[1]
fs = 96000
S = dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0)
st = oracle.eq_struct(fs, S)
x16 = oracle.quantize(synth.mix_like(fs * 30, fs, 2, seed=5))
(x16[:, 0].astype(np.float32) / np.float32(32768)).astype(np.float64).tofile(w + '/x.bin')
np.array(list(st.kind), np.float64).tofile(w + '/kinds.bin')
np.array(list(st.gain_db)).tofile(w + '/gdb.bin')
np.array(list(st.g)).tofile(w + '/g.bin')
np.array([[st.coef[i][k] for k in range(24)] for i in range(4)]).tofile(w + '/coef.bin')
PY
g++ -O2 -o "$W/emu" scripts/scan_precision_emu.cpp
cd "$W"
./emu 128 2 0; ./emu 128 0 0; ./emu 128 0 1; ./emu 128 1 1
