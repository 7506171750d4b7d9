#!/bin/bash
# Round 4: full SQ / TCC counter passes of the dominant kernel at HEAD, C3 625-trial shard
# and C2 (scripts/pmc.sh: one rocprofv3 --pmc run per counter set).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r04_pmc_c3_625 bash scripts/pmc.sh --config C3 --scaling strong --shard 8 --no-c3-strong --no-acc-f64 || exit $?
TAG=r04_pmc_c2 bash scripts/pmc.sh --no-c3-strong --no-acc-f64 || exit $?
