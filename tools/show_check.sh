#!/bin/bash
# Print what tools/gpu_check.sh TAG left under gpurun_out/TAG (CPU side).
O=gpurun_out/${1:-chk}
tail -1 $O/t.log
for i in 1 2; do
    python3 -c "import json; d=json.load(open('$O/b$i.json')); k=d['kernels_ms']; print(d['value'], d['ms_per_step'], 'bwd', k['grid_encode_backward'], 'fwd', k['grid_encode_forward'], 'frac', d['roofline']['frac'])"
done
python3 -c "
import json; s=json.load(open('$O/step.json')); k=s.get('kernels_us_per_step'); print(s.get('kernel_busy_us_per_step'), k)"
