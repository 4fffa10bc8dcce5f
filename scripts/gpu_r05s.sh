# round 5: active-band envelope tables -- the table-2 segment floor at C3, and C4 / C5 against the 3-band table
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="--steps 40 --warmup 5 --soak 0 --no-cpu-baseline --no-other-configs --no-pipeline"
prof() { timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05s_prof -o $1 --output-format csv -- python3 bench.py $2 $P > gpurun_out/r05s_$1.log 2>&1; }
prof c3_default "--config c3" || exit 1
AMX_ENV_LEMIN2=1024 prof c3_le1024 "--config c3" || exit 1
AMX_ENV_LEMIN2=1152 prof c3_le1152 "--config c3" || exit 1
AMX_ENV_BANDTAB=0 prof c3_tab3 "--config c3" || exit 1
prof c5_default "--config c5" || exit 1
AMX_ENV_BANDTAB=0 prof c5_tab3 "--config c5" || exit 1
prof c4_default "--config c4" || exit 1
AMX_ENV_BANDTAB=0 prof c4_tab3 "--config c4" || exit 1
