# round 4: HBM traffic per kernel (two PMC passes) for C3 and for C3 settings at 44.1 kHz is
# not a bench config -- C3 only, refreshed on the round-4 tree
set -o pipefail
CFG=c3 bash scripts/gpu_traffic.sh
