cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r04m
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r04m/a -o kt --output-format csv -- python3 -c "import torch; x=torch.ones(1000,device='cuda'); print(float(x.sum().cpu()))" > gpurun_out/r04m/a.log 2>&1; echo "torch-only rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r04m/b -o kt --output-format csv -- python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04m/b.log 2>&1; echo "smoke rc=$?"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r04m/c -o kt --output-format csv -- python3 -c "
import sys; sys.path[:0]=['djy-keto_amd']
import keto_mi355x as km, numpy as np
from keto_mi355x import synth
wl = synth.nested_groups(n_tuples=100000, seed=1) if hasattr(synth,'nested_groups') else None
print('lib only ok')" > gpurun_out/r04m/c.log 2>&1; echo "lib-import rc=$?"
find gpurun_out/r04m -name "*memory_copy*" | head
