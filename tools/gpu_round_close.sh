#!/bin/bash
# Round close-out evidence on the GPU box: smoke, the full GPU suite, rocprofv3 passes of the bench
# (kernel trace, FETCH_SIZE, WRITE_SIZE; tools/prof_r4.sh) and of LocalBA, the SQ counter passes
# (tools/pmc_kernel.sh), then the default bench line.  Every GPU step under its own time limit; the
# script stops at the first failure.  Post-processing on the CPU side:
#   tools/rocprof_stages.py  gpurun_out/close/prof/trace/.../run_kernel_stats.csv HEAD  > profiles/rNN_rocprof_stages.json
#   tools/traffic_json.py    gpurun_out/close/prof HEAD 256                              > profiles/traffic.json
#   tools/ba_traffic.py      gpurun_out/close/prof/ba 10 HEAD                          > profiles/rNN_localba_traffic.json
#   tools/sq_summary.py      gpurun_out/close/pmc                                      > profiles/rNN_sq_counters.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=${CLOSE_OUT:-gpurun_out/close}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1
rc=$?; echo rc=$rc >> $O/gputest.log; [ $rc -eq 0 ] || { tail -30 $O/gputest.log; exit $rc; }
tail -2 $O/gputest.log
OUT=$O/prof bash tools/prof_r4.sh > $O/prof.log 2>&1 || exit 1
OUT=$O/pmc bash tools/pmc_kernel.sh > $O/pmc.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 400 $O/bench.json
