# Span sync variants: LDS-staged words vs global words (tools/variants/libv_stage.so / libv_glob.so)
# at G = 2, 4, 8 on hard 1080p and 4K / 1080p scenes (resident JPEG stages).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for lib in stage glob; do
  for g in 2 4 8; do
    for sc in "1080p hard" "4k scene" "1080p scene"; do
      set -- $sc
      VF_JPEG_SYNC=pass VF_JPEG_SYNC_G=$g VFILTER_LIB=$PWD/tools/variants/libv_$lib.so timeout -k 10 200 python3 tools/jpeg_bench.py --sizes $1 --content $2 --batch 32 --iters 8 --cpu-seconds 0 --resident-only > gpurun_out/sl.jsonl 2> gpurun_out/sl.log || { echo RUN_FAILED; tail -20 gpurun_out/sl.log; exit 1; }
      python3 -c "
import json
d = json.loads(open('gpurun_out/sl.jsonl').read().splitlines()[-1]); s = d['stages_ms']
print('rep $rep $lib G$g', d['size'], d['content'], d['gpu_resident_fps'], d['parity_vs_oracle'], 'sync', s['huffman_sync'])"
    done
  done
done
done
