set -eo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
for i in 1 2; do
  for a in "--steps 20 --warmup 5 --graph-steps 1" "--steps 20 --warmup 5 --graph-steps 4" "--steps 20 --warmup 5 --graph-steps 10" "--steps 20 --warmup 5 --graph-steps 20" "--steps 50 --warmup 20 --graph-steps 1" "--steps 50 --warmup 20 --graph-steps 8"; do
    timeout -k 10 200 python -u bench.py --no-cpu $a > $O/x.json 2> $O/x.err
    python -c "import json; d=json.load(open('$O/x.json')); print('$i', '$a', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
  done
done
