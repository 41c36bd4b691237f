#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
OUT=gpurun_out/r5m_pmc bash tools/pmc_kernel.sh
python3 tools/sq_summary.py gpurun_out/r5m_pmc > gpurun_out/r5m_sq.json
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r5m_sq.json'))
ks=d.get('kernels',d)
for k,v in ks.items():
    if 'resize' in k or 'blur' in k: print(k, json.dumps(v))
PY
