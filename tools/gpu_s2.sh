#!/bin/bash
# host-issue profile of the metric step (is the host the bottleneck in the short-kernel phases?)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s2
mkdir -p $O
cd $R
timeout -k 10 400 python tools/host_issue_profile.py > $O/host.log 2>&1 || { echo FAIL host; tail -30 $O/host.log; exit 1; }
head -120 $O/host.log
