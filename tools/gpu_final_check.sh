#!/bin/bash
# smoke(), the full GPU suite and the default bench line at the current tree (round-end rehearsal)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/fin3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin3/smoke.log 2>&1 || { tail -20 gpurun_out/fin3/smoke.log; exit 1; }
tail -1 gpurun_out/fin3/smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/fin3/gputest.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/fin3/gputest.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/fin3/gputest.log; exit $rc; }
tail -2 gpurun_out/fin3/gputest.log
timeout -k 10 600 python bench.py > gpurun_out/fin3/bench.json 2> gpurun_out/fin3/bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/fin3/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['localba']['iters_per_s'], d['stage_ms_per_step'])"
