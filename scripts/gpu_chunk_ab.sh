set -u
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
for c in 128 256 512; do
  GFD_HUB_CHUNK=$c timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 10 > gpurun_out/chunk_$c.json 2> gpurun_out/chunk_$c.err
  rc=$?; echo "chunk $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/chunk_$c.json')); print('$c', round(d['ms_per_step'],3), {k: round(x['ms'],3) for k,x in d['kernels'].items()})"
done
