#!/bin/bash
# round profile of the three bench workloads (tools/profile_bench.sh each); first failure ends it
set -o pipefail
TAG=${1:-r02_v3}
for W in ${WORKLOADS:-adanalytics ssb highcard index}; do
  bash tools/profile_bench.sh $TAG $W 10 || exit 1
done
