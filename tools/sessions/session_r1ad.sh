#!/bin/bash
# L96 halos: DPP with interior-first RHS order vs ds_swizzle (LDS pipe) with the same order.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "scan_dpp:300:python tools/lanes_scan.py 65536 40 2000 > gpurun_out/scan_dpp.txt" \
  "scan_swz:300:IPMC_LIB_PATH=\$PWD/ip_mcmc_amd/lib_exp/libipmc.so python tools/lanes_scan.py 65536 40 2000 > gpurun_out/scan_swz.txt" \
  "par_swz:300:IPMC_LIB_PATH=\$PWD/ip_mcmc_amd/lib_exp/libipmc.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k 'l96 or sweep'"
