# round 5: the TrackStream replay segfault -- the test alone with the product library, then with the library before the fix-up rework
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -X faulthandler -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "track_stream" > gpurun_out/r05ad_cur.log 2>&1; echo "cur rc=$?"
AMX_LIB=audio-mastering-engine_amd/lib_var/libamx_prev.so timeout -k 10 300 python -u -X faulthandler -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "track_stream" > gpurun_out/r05ad_prev.log 2>&1; echo "prev rc=$?"
