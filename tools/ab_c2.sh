# C2 (2^22 fwd+inv NTT) through bench.py's side measurement for several library builds on one box
set -e
cd $GRAFT_REPO_ROOT
for lib in ab/libstarkgpu_e13.so ab/libstarkgpu_base.so zk-stark-tutor_amd/starkgpu/libstarkgpu.so; do
  echo "== $lib"
  SG_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_c2_tmp.log 2>&1
  python -c "
import json;d=json.loads(open('gpurun_out/ab_c2_tmp.log').read().strip().splitlines()[-1]); s=d['side']
print(d['prove_ms'], s['c2_ntt_fwd_inv_2p22_ms'], s['c5_ntt_2p27_ms'], s['north_star_lde_fri_commit_2p24_ms'])"
done
