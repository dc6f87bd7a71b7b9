# Run a command with a heartbeat file under gpurun_out/ (a long quiet phase must not look hung):
#   bash tools/hb.sh <command...>
mkdir -p gpurun_out
(while true; do date +%s > gpurun_out/heartbeat; sleep 20; done) &
HB=$!
trap "kill $HB 2>/dev/null || true" EXIT
"$@"
