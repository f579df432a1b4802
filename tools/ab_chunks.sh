#!/bin/bash
for c in 64 128 256 512; do echo "chunk $c"; MVS_TILE_CHUNK=$c timeout -k 10 120 python tools/ab_variants.py 0 2>&1 | grep -v amdgpu.ids; done
