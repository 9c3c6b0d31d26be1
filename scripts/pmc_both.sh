#!/bin/bash
# GPU-box step: SQ counter groups for the compress and the decompress kernel of one kind
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=pcc WHICH=compress bash scripts/pmc_compress.sh > gpurun_out/pcc.txt 2>&1 && \
TAG=pcd WHICH=decompress bash scripts/pmc_compress.sh > gpurun_out/pcd.txt 2>&1
rc=$?
cat gpurun_out/pcc.txt gpurun_out/pcd.txt | grep -v fill_kernel
exit $rc
