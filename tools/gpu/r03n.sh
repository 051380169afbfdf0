#!/bin/bash
# round 3 GPU check N: Kafka e2e legs, pinned vs floating serving threads
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 400 python -u tools/serve_probe/kafka_legs.py > $O/legs.out 2> $O/legs.err
echo "rc=$?"
cat $O/legs.out
echo ALLDONE
