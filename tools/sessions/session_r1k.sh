#!/bin/bash
# Halo experiment: DPP movs (default build) vs ds_bpermute (IPMC_HALO_LDS=1 build) for LPC 2/4.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
tools/gpu_session.sh \
  "scan_dpp:300:python tools/lanes_scan.py 65536 40 2000 > gpurun_out/scan_dpp.txt" \
  "scan_lds:300:IPMC_LIB_PATH=\$PWD/ip_mcmc_amd/lib_exp/libipmc.so python tools/lanes_scan.py 65536 40 2000 > gpurun_out/scan_lds.txt" \
  "scan_dpp2:300:python tools/lanes_scan.py 65536 40 2000 > gpurun_out/scan_dpp2.txt"
