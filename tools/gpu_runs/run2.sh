set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/quick_step.py --steps 4 > gpurun_out/q2.log 2>&1
rc=$?; echo "quick rc=$rc" >> gpurun_out/q2.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python3 tools/quick_step.py --steps 2 > gpurun_out/p2.log 2>&1
echo "prof rc=$?" >> gpurun_out/p2.log
