#!/bin/bash
# graph shapes probe (tools/graph_probe.hip) under the runtime's graph settings
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03_v19
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/graph_probe > $O/default.txt 2>&1; cat $O/default.txt
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 ./tools/graph_probe > $O/nocapture.txt 2>&1; cat $O/nocapture.txt
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 120 ./tools/graph_probe > $O/queues4.txt 2>&1; cat $O/queues4.txt
