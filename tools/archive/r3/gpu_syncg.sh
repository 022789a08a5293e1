# Span sync (k_syncg) on the GPU: JPEG tests (default G = 4), then the resident JPEG stages for
# G = 0 (host-looped k_sync), 1, 2, 4, 8 on hard 1080p and 4K scenes, and the pass path against the
# speculative one on 1080p / 480p scenes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sg_pytest_jpeg.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -40 gpurun_out/sg_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/sg_pytest_jpeg.log
run() {  # name env... -- args
  local name=$1; shift
  local e=(); while [ "$1" != "--" ]; do e+=("$1"); shift; done; shift
  env "${e[@]}" timeout -k 10 200 python3 tools/jpeg_bench.py --batch 32 --iters 10 --cpu-seconds 0 --resident-only "$@" > gpurun_out/sg_$name.jsonl 2> gpurun_out/sg_$name.log || { echo RUN_FAILED $name; tail -20 gpurun_out/sg_$name.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/sg_$name.jsonl'):
    d = json.loads(l); s = d['stages_ms']
    print('$name', d['size'], d['content'], d['gpu_resident_fps'], d['parity_vs_oracle'], 'sync', s['huffman_sync'], 'write', s['huffman_write'], 'passes', s.get('sync_passes'))"
}
for g in 0 1 2 4 8; do run hard_g$g VF_JPEG_SYNC_G=$g -- --sizes 1080p --content hard || exit 1; done
for g in 0 4 8; do run k4_g$g VF_JPEG_SYNC_G=$g -- --sizes 4k || exit 1; done
run s_spec VF_JPEG_SYNC=spec -- --sizes 480p,1080p || exit 1
for g in 1 2 4 8; do run s_pass_g$g VF_JPEG_SYNC=pass VF_JPEG_SYNC_G=$g -- --sizes 480p,1080p || exit 1; done
GS="4 8" bash tools/r3/gpu_syncg_trace.sh
# k_syncg counters (tools/build_syncg_stats.sh) on hard 1080p and 4K scenes, G = 4 and 8.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 4 8; do
  for sc in "1080p hard" "4k scene"; do
    set -- $sc
    VF_SYNCG_STATS=1 VF_JPEG_SYNC_G=$g VFILTER_LIB=$PWD/tools/variants/libv_syncg_stats.so timeout -k 10 200 python3 tools/jpeg_bench.py --sizes $1 --content $2 --batch 32 --iters 2 --cpu-seconds 0 --resident-only > gpurun_out/sgs_${g}_$1.log 2>&1 || { echo STATS_FAILED; tail -20 gpurun_out/sgs_${g}_$1.log; exit 1; }
    echo "G $g $1 $2"; grep "\[syncg\]" gpurun_out/sgs_${g}_$1.log | tail -4
  done
done
