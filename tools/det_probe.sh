#!/bin/bash
set -u
O=gpurun_out/${1:-det_probe}; mkdir -p $O
for v in "cl bench0" "cl bench1" "nchw bench0" "nchw bench1" "cl bench1 fp32"; do
  timeout -k 10 300 python3 tools/det_probe.py $v >> $O/probe.txt 2> $O/probe_$(echo $v | tr ' ' _).err || exit 1
done
cat $O/probe.txt
