# JPEG system leg with 1 / 2 / 4 worker processes on one card, short time limits, stderr kept.
set -o pipefail
mkdir -p gpurun_out
for w in 1 2 4; do
  timeout -k 10 90 python3 -u tools/pipeline_bench.py --workers $w --gpus 1 --jpeg --size 1080p --batch 32 --policy pull \
      --frames $((6144 * w)) > gpurun_out/r6_mw_$w.json 2> gpurun_out/r6_mw_$w.err
  rc=$?
  echo "workers $w rc $rc"; tail -c 600 gpurun_out/r6_mw_$w.json; echo; tail -5 gpurun_out/r6_mw_$w.err
  [ $rc -ne 0 ] && break
done
exit 0
