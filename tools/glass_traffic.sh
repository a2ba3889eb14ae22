set -e
export TMPDIR=/tmp
for v in tree:raytracingengine_amd/librtamd.so wf3:tools/variants/wf3.so; do
  name=${v%%:*}; lib=${v#*:}
  O=gpurun_out/r04h/traffic_$name
  mkdir -p $O
  RTAMD_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p1 -o pmc -- python3 tools/profile_kernel.py glass 10 > $O/p1.log 2>&1
  RTAMD_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p2 -o pmc -- python3 tools/profile_kernel.py glass 10 > $O/p2.log 2>&1
  python3 tools/pmc_summary.py $O > /dev/null
  echo done $name
done
