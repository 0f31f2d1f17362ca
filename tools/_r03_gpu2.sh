#!/bin/bash
set -o pipefail
timeout -k 10 200 python -u tools/_nan_probe.py > gpurun_out/nan_probe.log 2>&1 || exit 1
bash tools/_r03_gpu1.sh
