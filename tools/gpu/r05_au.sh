#!/bin/bash
# round 5, call AU: full verification of the round's final build (GPU suite, smoke, bench, round profile)
set -o pipefail
OUT=r05v8 bash tools/gpu/r05_verify.sh
