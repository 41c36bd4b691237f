mkdir -p gpurun_out
ORBX_LIB_OVERRIDE=$PWD/build_ab/fprobe/liborbx.so timeout -k 10 200 python tools/fast_probe.py > gpurun_out/fast_probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/fast_probe.log
