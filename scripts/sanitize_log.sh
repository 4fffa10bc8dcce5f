# Host ASan + UBSan runs of the FLAC decoder and the C oracle (tests/test_sanitize.py),
# the log committed as profiles/r05_sanitize.log.  CPU only.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
{ echo "# $(date -u +%FT%TZ)  g++ $(g++ -dumpfullversion)  gcc $(gcc -dumpfullversion)"
  python -m pytest tests/test_sanitize.py tests/test_flac.py tests/test_oracle.py -v -s -p no:cacheprovider 2>&1
} > profiles/r05_sanitize.log
