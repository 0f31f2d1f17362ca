#!/bin/bash
# round 5, call AR: full verification of the build with tile form 4 by size (GPU suite, smoke, bench, round profile)
set -o pipefail
OUT=r05v7 bash tools/gpu/r05_verify.sh
