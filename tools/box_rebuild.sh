#!/bin/bash
# GPU call (round 6): rebuild every HIP source ON THE GPU BOX from this tree (build --force:
# hipcc gfx950 there, not the prebuilt librtamd.so that travelled), record what was built, then
# run the GPU suite and the driver-shaped bench line with that library.
set -eu
export TMPDIR=/tmp
OUT=gpurun_out/box_rebuild
mkdir -p $OUT
sha256sum raytracingengine_amd/librtamd.so > $OUT/prebuilt.sha256
( time timeout -k 10 900 python -m raytracingengine_amd.build --force ) > $OUT/build.txt 2>&1
sha256sum raytracingengine_amd/librtamd.so > $OUT/rebuilt.sha256
python -c "
import json, os
from raytracingengine_amd import capi, build as B
i = capi.build_info()
i['tree_digest'] = B.source_digest()
i['lib_mtime'] = os.path.getmtime(B.LIB)
print(json.dumps(i, indent=1))" > $OUT/build_info.json
cat $OUT/build_info.json
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread \
  > $OUT/gpu_tests.txt 2>&1
tail -n 2 $OUT/gpu_tests.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err
python -c "
import json; d = json.load(open('$OUT/bench_s20.json'))
print(d['value'], d['ms_per_step'], d['build'], d['parity'])"
