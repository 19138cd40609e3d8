set -u
export TMPDIR=/tmp
SWEEP="1,1024,1;1,512,1;1,256,1;1,256,2;1,256,4;1,512,2;1,1024,2" timeout -k 10 300 python -u tools/sweep.py 16 > gpurun_out/sweep_e16.log 2>&1 || exit $?
SWEEP="1,256,4;1,256,8;1,512,2;1,512,4;1,1024,2" timeout -k 10 200 python -u tools/sweep.py 14 15 > gpurun_out/sweep_e14.log 2>&1 || exit $?
TSPGPU_LDS_TABLE_MAX_N=0 SWEEP="1,256,4;1,256,8;1,256,2" timeout -k 10 200 python -u tools/sweep.py 12 > gpurun_out/sweep_e12.log 2>&1 || exit $?
cat gpurun_out/sweep_e*.log
