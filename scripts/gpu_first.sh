#!/bin/bash
# first GPU check: torch.mm out_dtype support, kernels vs oracle, smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "
import torch
a=torch.randn(64,256,device='cuda',dtype=torch.bfloat16); b=torch.randn(256,512,device='cuda',dtype=torch.bfloat16)
c=torch.mm(a,b,out_dtype=torch.float32); print('mm out_dtype ok', c.dtype, (c-(a.float()@b.float())).abs().max().item())
o=torch.empty(64,512,device='cuda'); torch.mm(a,b,out_dtype=torch.float32,out=o); print('mm out= ok', (o-c).abs().max().item())
print(torch.cuda.get_device_name(0))
" > gpurun_out/first_mm.log 2>&1; echo "mm rc=$?"
timeout -k 10 600 python -m pytest tests/test_gpu_model.py -x -q > gpurun_out/first_pytest.log 2>&1; echo "pytest rc=$?"
tail -40 gpurun_out/first_pytest.log
