#!/bin/bash
# r03ar: attributed PMC passes (tools/pmc_kernels.sh) of the final build: LightGlue stage and ViT forward
set -u
timeout -k 10 900 bash tools/pmc_kernels.sh r03ar
