#!/bin/bash
# round-6 session g: P1 knockouts (timing only, wrong streams): counters + stamps
set -uo pipefail
bash tools/var_sq.sh r06_g "base koq kos" || exit $?
