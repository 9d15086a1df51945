#!/bin/bash
cd $GRAFT_REPO_ROOT
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests/test_trainer_gpu.py tests/test_model_gpu.py -x -q -m gpu > gpurun_out/t6.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t6.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b6.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b6.log; ok $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-overlap > gpurun_out/b6_noov.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b6_noov.log; ok $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/p6.log 2>&1; echo "prof rc=$?" >> gpurun_out/p6.log
