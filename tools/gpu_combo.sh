#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_narrow.sh && bash tools/gpu_attn41.sh
