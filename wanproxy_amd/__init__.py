"""wanproxy_amd: an MI355X-native XCodec dedup engine (HIP kernels for gfx950
behind the C ABI of include/xcgpu.h).  See DESIGN.md."""
__all__ = ['xcgpu', 'synth', 'build']
