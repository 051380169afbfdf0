#!/bin/bash
# round 3 GPU check L: Kafka e2e legs (echo vs GPU scorer), small-batch counters with the final kernel
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 300 python -u tools/serve_probe/kafka_legs.py > $O/legs.out 2> $O/legs.err; echo "legs rc=$?"
cat $O/legs.out
cd /tmp
for mode in mb32 mb100; do
  for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
              "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    tag=$(echo $pass | cut -c4-9)
    timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex ae_minibatch \
      -d "$GRAFT_REPO_ROOT/$O/${mode}_$tag" -o run --pmc $pass -- python3 "$GRAFT_REPO_ROOT/tools/pmc_small.py" $mode \
      > "$GRAFT_REPO_ROOT/$O/${mode}_$tag.log" 2>&1 || { echo "pmc $mode rc=$?"; exit 1; }
    echo "== pmc $mode $tag ok"
  done
done
echo ALLDONE
