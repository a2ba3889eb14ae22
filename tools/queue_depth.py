import sys, time; sys.path.insert(0,'.')
import bench
args = bench.parse_args(["--no-cpu-baseline"])
R = bench.Runner(args)
from raytracingengine_amd.configs import make_config
sc = make_config("c2", aa=1)
for depth in (2, 3, 4, 2):
    el = bench.pipelined_frames(R, sc, 200, 20, depth, 1)
    print(depth, round(el / 200 * 1e6, 2), "us/frame", flush=True)
res = bench.frames_mode(R, sc, 200, 20, "f64", 1, 0)
print("serial", round(res["elapsed"] / 200 * 1e6, 2), "us/frame")
