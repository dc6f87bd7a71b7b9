# The GPU suite with every alternate path forced at once (each is a default's A/B knob; the proofs
# and roots must not depend on any of them).  Since round 6 the product library reads none of these
# (csrc/knobs.hpp): the suite loads the A/B build (make -C zk-stark-tutor_amd ab) via SG_LIB_PATH,
# which reads them at context creation / first use:
#   SG_NO_DOMAIN_CACHE=1          public domain/AIR tables recomputed per proof
#   SG_AIR_GENERIC=1              the Rescue AIR through its expanded groups
#   SG_NTT_TILES=0                three-pass NTTs on 2048-element tiles at every size
#   SG_GEO_DECIMATE=0             full-group geometric interpolation
#   SG_STREAM_PRIORITY=0          default HIP stream priorities
#   SG_DIST_FRI_TAIL=0            every sharded FRI round sharded (no hand-over)
#   SG_MERKLE_QUAD_LEAF_BELOW=0   one lane per leaf at every leaf level
#   SG_MERKLE_QUAD_TOP=0          64-node quad blocks only at tree tops
#   SG_MERKLE_LEAF_PAIRS=0        one leaf per lane in the throughput-bound leaf kernel
#   SG_MERKLE_NODE_FUSE=3         three node levels per launch (round 3's plan)
#   SG_NTT_SMALL_WHOLE=0          small transforms as bit-reversal gather + generic pass
#   SG_MERKLE_FOREST_QUAD=0       forests' node levels through the one-lane-per-node kernel (round 4)
#   SG_LEAN_TREES=0               the prove's retained trees keep their leaf digests (round 4)
#   SG_MERKLE_QUAD_LEAF_NODES=64  64-leaf quad blocks for latency-bound leaf levels
#   SG_MERKLE_QUAD_TOP_MAX=64     one-block tree tops only from 64 nodes down
#   SG_FRI_GATE=0                 each FRI round launched after its challenge (no device gate; round 6)
#   SG_TAIL_DIRECT=0              the proof tail serialized to device memory and copied (round 6)
#   SG_FRI_TWO_STREAMS=0          gated FRI rounds all on the main stream (round 6)
# Usage (from the repo root on the GPU box): bash tools/gpu_alt_paths.sh [tag]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-alt}
cd "$R"
mkdir -p gpurun_out
SG_LIB_PATH=$R/zk-stark-tutor_amd/starkgpu/libstarkgpu_ab.so \
SG_NO_DOMAIN_CACHE=1 SG_AIR_GENERIC=1 SG_NTT_TILES=0 SG_GEO_DECIMATE=0 SG_STREAM_PRIORITY=0 SG_DIST_FRI_TAIL=0 \
SG_MERKLE_QUAD_LEAF_BELOW=0 SG_MERKLE_QUAD_TOP=0 SG_MERKLE_LEAF_PAIRS=0 SG_MERKLE_NODE_FUSE=3 SG_NTT_SMALL_WHOLE=0 \
SG_MERKLE_FOREST_QUAD=0 SG_LEAN_TREES=0 SG_MERKLE_QUAD_LEAF_NODES=64 SG_MERKLE_QUAD_TOP_MAX=64 SG_FRI_GATE=0 SG_TAIL_DIRECT=0 SG_FRI_TWO_STREAMS=0 \
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pt_alt_$TAG.log 2>&1
