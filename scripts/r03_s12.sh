#!/bin/bash
# Coverage step: one launch per step vs the two-stream split on the working tree, interleaved.
set -e
for i in 1 2 3; do
  STREAMS=1 timeout -k 10 200 python scripts/time_cov.py one
  STREAMS=2 timeout -k 10 200 python scripts/time_cov.py split
done
