# A/B: the two-pixel blend held to 64 VGPRs (8 waves per SIMD instead of 7).
p = "gs_kernels.hip"
s = open(p).read()
a = "__global__ __launch_bounds__(64 * GS_PX2_WPG) void gs_blend_px2_kernel(FrameParams fp, Buffers b) {"
assert s.count(a) == 1
s = s.replace(a, "__global__ __launch_bounds__(64 * GS_PX2_WPG) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_blend_px2_kernel(FrameParams fp, Buffers b) {")
open(p, "w").write(s)
