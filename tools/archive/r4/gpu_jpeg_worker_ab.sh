# The JPEG worker form (one thread, three batches in flight: tools/jpeg_modes.py async3) with
# VAR=A and VAR=B, alternating, three reps:  bash tools/r4/gpu_jpeg_worker_ab.sh VAR A B [size]
set -o pipefail
VAR=$1; A=$2; B=$3; SIZE=${4:-1080p}
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 120 python3 tools/jpeg_modes.py $SIZE async3 > gpurun_out/wab.json 2> gpurun_out/wab.err || { echo WORKER_AB_FAILED; tail -20 gpurun_out/wab.err; exit 1; }
    echo "$VAR=$v rep $rep $(tail -1 gpurun_out/wab.json)"
  done
done
