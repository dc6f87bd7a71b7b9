# Same-box interleaved A/B runner (one script for every experiment; the round-2 per-experiment
# tools/ab_*.sh scripts are folded into it -- their logs stay under profiles/r02_ab_*.log).
#
#   bash tools/ab.sh MEASURE ROUNDS VARIANT [VARIANT ...]
#
# MEASURE  prove[:STEPS[:LOG]]  tools/step_timing.py   ms per Stark::prove (trace 2^LOG, default 20)
#          c2[:LOG]             tools/c2_time.py       fwd+inv NTT of 2^LOG (default 22)
#          merkle[:LOG]         tools/bench_merkle.py  Merkle tree of 2^LOG leaves (default 25)
#          ntt[:LOG]            tools/bench_ntt.py     NTT passes of 2^LOG (default 22)
#          bench                bench.py --no-cpu-baseline --steps 3 --warmup 1 (prove, C2, C5, 2^24 block)
#          dist[:STEPS[:LOG]]   tools/dist_prove_time.py  sharded prove on a one-rank RCCL communicator
#          c5dist[:LOG]         tools/c5_dist_time.py     four-step NTT of 2^LOG on a one-rank communicator
# VARIANT  LABEL or LABEL=K1=V1,K2=V2: environment of that variant; the key `lib` names a library
#          build (path relative to the repo root) loaded through SG_LIB_PATH, e.g.
#            base=lib=ab/libstarkgpu_base.so  new  fuse3=SG_MERKLE_NODE_FUSE=3
# Each round runs every variant once, in order; each run prints "LABEL: <last line of its output>".
# Every run has its own time limit; a failing run stops the script (set -e).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
MEASURE=${1:?measure}
ROUNDS=${2:?rounds}
shift 2
IFS=: read -r KIND A1 A2 <<< "$MEASURE"
PICK=""
case "$KIND" in
  prove)  CMD=(python tools/step_timing.py "${A1:-8}" "${A2:-20}"); LIMIT=200 ;;
  c2)     CMD=(python tools/c2_time.py "${A1:-22}"); LIMIT=120 ;;
  merkle) CMD=(python tools/bench_merkle.py "${A1:-25}"); LIMIT=120; PICK="ms/build" ;;
  ntt)    CMD=(python tools/bench_ntt.py "${A1:-22}"); LIMIT=120 ;;
  dist)   CMD=(python tools/dist_prove_time.py "${A1:-5}" "${A2:-20}" sharded_world1); LIMIT=200 ;;
  c5dist) CMD=(python tools/c5_dist_time.py "${A1:-27}"); LIMIT=200 ;;
  bench)  CMD=(python bench.py --no-cpu-baseline --steps 3 --warmup 1); LIMIT=300 ;;
  *) echo "unknown measure $KIND" >&2; exit 2 ;;
esac
for ((round = 1; round <= ROUNDS; round++)); do
  for V in "$@"; do
    LABEL=${V%%=*}
    ENVS=()
    if [[ "$V" == *=* ]]; then
      IFS=, read -ra KV <<< "${V#*=}"
      for kv in "${KV[@]}"; do
        if [[ "$kv" == lib=* ]]; then ENVS+=("SG_LIB_PATH=$R/${kv#lib=}"); else ENVS+=("$kv"); fi
      done
    fi
    if [ -n "$PICK" ]; then
      OUT=$(env "${ENVS[@]}" timeout -k 10 $LIMIT "${CMD[@]}" 2>&1 | grep -m1 "$PICK")
    else
      OUT=$(env "${ENVS[@]}" timeout -k 10 $LIMIT "${CMD[@]}" 2>&1 | tail -n 1)
    fi
    echo "$LABEL: $OUT"
  done
done
