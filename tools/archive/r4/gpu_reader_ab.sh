# Round-4 A/B of the stdlib transport's readers (VF_TCP_READER=thread: one thread per peer
# connection; select: one select loop per listener): the control plane alone
# (tools/distributor_overhead.py --no-copy, 1 / 2 / 4 / 8 echo workers, JPEG-size frames and the
# mixed configs[3] stream), then the JPEG system leg with one GPU worker.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/reader_ab.jsonl
rm -f $OUT
for r in thread select; do
  for n in 1 2 4 8; do
    VF_TCP_READER=$r timeout -k 10 120 python -u tools/distributor_overhead.py --no-copy --workers $n --policy pull --bytes 181876 --batch 32 --frames $((8000 * n)) --group 16 --out gpurun_out/rab_one.jsonl > /dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/rab_one.jsonl').read().splitlines()[-1]); d['reader']='$r'; print('$r', d['workers'], d['frame_bytes'], d['fps'], d['distributor_cpu_us_per_frame']); open('$OUT','a').write(json.dumps(d)+'\n')"
    VF_TCP_READER=$r timeout -k 10 120 python -u tools/distributor_overhead.py --no-copy --workers $n --policy pull --mixed --batch 16 --frames $((4000 * n)) --group 8 --out gpurun_out/rab_one.jsonl > /dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/rab_one.jsonl').read().splitlines()[-1]); d['reader']='$r'; print('$r', d['workers'], d['frame_bytes'], d['fps'], d['distributor_cpu_us_per_frame']); open('$OUT','a').write(json.dumps(d)+'\n')"
  done
  VF_TCP_READER=$r timeout -k 10 150 python -u tools/pipeline_bench.py --jpeg --size 1080p --batch 32 --policy pull --frames 16384 > gpurun_out/rab_pipe.json 2> gpurun_out/rab_pipe.err || { echo PIPE_FAILED; tail -20 gpurun_out/rab_pipe.err; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/rab_pipe.json').read().splitlines()[-1]); print('$r system jpeg', r['fps'], r['n_errors'])"
done
echo READER_AB_OK
