import sys; sys.path.insert(0,'.')
import torch
from raytracingengine_amd import capi
from raytracingengine_amd.configs import make_config
ctx=capi.Context(0); s=torch.cuda.Stream(); ctx.set_stream(s.cuda_stream)
for name in ["mesh","bigmesh"]:
    sc=make_config(name); ds=ctx.scene(sc); W,H=sc.camera.width,sc.camera.height
    h=torch.empty(W*H*3,dtype=torch.float64,device="cuda")
    for fl in (0, capi.RT_FLAG_NO_BVH):
        o=capi.default_opts(tonemap=-1, flags=fl|capi.RT_FLAG_TIME_KERNEL)
        ds.render_device(h.data_ptr(),None,None,o); ctx.reset_stats()
        for _ in range(3): ds.render_device(h.data_ptr(),None,None,o)
        st=ctx.stats(); print(name, "bvh" if fl==0 else "all-triangles", "%.3f ms"%(st.kernel_ms/st.launches), flush=True)
    ds.close()
