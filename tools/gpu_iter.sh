#!/bin/bash
# One iteration on the GPU box: the named test files, probes, then same-box
# bench A/B legs of an env knob. usage (on the box):
#   bash tools/gpu_iter.sh TAG "tests/a.py tests/b.py" "KNOB1 KNOB2"
set -eo pipefail
TAG=$1; TESTS=$2; KNOBS=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
fi
for probe in ${PROBES:-}; do
  timeout -k 10 200 python -u tools/$probe.py > $O/$probe.json 2> $O/$probe.err
done
# a knob "A+B" sets both A and B to the value
for KNOB in $KNOBS; do
  for rep in 1 2; do
    for v in 0 1; do
      ENVS=""
      for K in ${KNOB//+/ }; do ENVS="$ENVS $K=$v"; done
      env $ENVS timeout -k 10 200 python -u bench.py --no-cpu --no-legs --no-dp-path --no-render --steps 200 \
          > $O/ab_${KNOB}_${v}_${rep}.json 2> $O/ab_${KNOB}_${v}_${rep}.err
    done
  done
done
