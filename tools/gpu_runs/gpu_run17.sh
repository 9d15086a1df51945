#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_wgrad.py --only gate_up,lm_head --cfgs 1,3,5,6 > gpurun_out/bw17.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/bw17.log
