import sys; sys.path[:0]=['/root/repo/real-time-opencl-raytracer_amd','/root/repo']
import rtamd, torch
r = rtamd.Renderer(0)
m = rtamd.Mesh.cornell(); r.upload(rtamd.Scene.from_mesh(m, m.build_sbvh()))
cus = torch.cuda.get_device_properties(0).multi_processor_count
for n in [1, 4, 16, 64, 256, 1024, 4096, 16384, 65536, 262144, 1048576]:
    ms, recs = r.gather_peak(n, 256)
    rps = recs / (ms * 1e-3)
    print(f"table {n:8d} rec ({n*64/1024:9.1f} KiB): {cus/rps*1e9:6.3f} ns/rec/CU  lane-bytes {rps*56/1e12:6.2f} TB/s")
