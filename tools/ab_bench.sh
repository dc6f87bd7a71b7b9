# same-box A/B of the headline bench: round-1 library (ab/libstarkgpu_head.so) vs the current one
# and twiddle-plan variants; prints prove_ms, the workload NTT rate and the side measurements
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  echo "== $1" >> gpurun_out/ab_bench.log
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/ab_tmp.log 2>&1
  python -c "
import json;d=json.loads(open('gpurun_out/ab_tmp.log').read().strip().splitlines()[-1]); s=d['side']
print(d['prove_ms'], d.get('ntt',{}).get('ntt_gelem_s'), s['c2_ntt_fwd_inv_2p22_ms'], s['c5_ntt_2p27_ms'], s['c4_prove_trace_2p16_ms'], s['north_star_lde_fri_commit_2p24_ms'])" >> gpurun_out/ab_bench.log
}
rm -f gpurun_out/ab_bench.log
for v in ${AB_VARIANTS:-head new table head new table}; do
  case $v in
    head) run head "SG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libstarkgpu_head.so" ;;
    new) run new "SG_X=1" ;;
    table) run table_only "SG_NTT_TWCUT=40" ;;
    top2) run top2 "SG_NTT_TWTOP=2" ;;
    top4) run top4 "SG_NTT_TWTOP=4" ;;
    prev) run prev "SG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libstarkgpu_prev.so" ;;
    cur) run cur "SG_X=1" ;;
  esac
done
