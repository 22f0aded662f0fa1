#!/bin/bash
# FETCH/WRITE bytes of k_integrate per timing probe (SEMTSDF_DEBUG_INTEGRATE)
set -u
for d in ${1:-0 3 4 10}; do
  SEMTSDF_DEBUG_INTEGRATE=$d bash tools/pmc_groups.sh gpurun_out/trd/d$d FETCH_SIZE WRITE_SIZE > /dev/null || exit 1
  python3 tools/traffic.py gpurun_out/trd/d$d "k_integrate<true, true, false, false, false, false, true>" gpurun_out/trd/d$d.json 512 > /dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/trd/d$d.json')); print('debug $d: fetch %.1f MB (raw %.1f) write %.1f MB' % (d['fetch_bytes']/1e6, d['fetch_size_kib_raw']*1024/1e6, d['write_bytes']/1e6))"
done
