#!/bin/bash
# round-6 close on the final build: suite B + smoke, then suite A
cd "$(dirname "$0")/../.."
bash tools/gpu/run_r6_final_b.sh && bash tools/gpu/run_r6_final_a.sh
