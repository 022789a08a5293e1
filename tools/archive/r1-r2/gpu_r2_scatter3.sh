# A/B: JPEG results scattered into ring slots (1) vs copied by the worker loop (0), 480p + 1080p, twice
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_sc3_pipe.jsonl
for r in 1 2; do
for sc in 1 0; do
for size in 480p 1080p; do
echo "{\"VF_JPEG_SCATTER\": $sc}" >> gpurun_out/r2_sc3_pipe.jsonl
VF_JPEG_SCATTER=$sc timeout -k 10 200 python -u tools/pipeline_bench.py --jpeg --workers 1 --gpus 1 --size $size --batch 32 --frames 16384 --policy pull --out gpurun_out/r2_sc3_pipe.jsonl > gpurun_out/r2_sc3_pipe.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_sc3_pipe.log; exit 1; }
done; done; done
python3 -c "
import json
sc = None
for l in open('gpurun_out/r2_sc3_pipe.jsonl'):
    d = json.loads(l)
    if 'VF_JPEG_SCATTER' in d: sc = d['VF_JPEG_SCATTER']; continue
    print('scatter', sc, d['size'], d['fps'], d['n_errors'])
"
