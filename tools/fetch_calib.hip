// fetch_calib.hip -- unit check of rocprofv3 FETCH_SIZE on gfx950 per load
// shape: each kernel reads exactly BYTES bytes once, fully coalesced (no
// re-read possible), so FETCH_SIZE * 1024 / BYTES is the counter's scale
// for that shape.  Shapes: 16 B/lane aligned (global_load_dwordx4), 16 B/lane
// at a 4-byte-aligned base (what the A4 address mode compiles to), and
// 4 B/lane (global_load_dword).  Run under rocprofv3 --pmc FETCH_SIZE.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr size_t BYTES = (size_t)1 << 30;

__global__ __launch_bounds__(256) void rd_x4(const uint8_t *p, size_t nvec, uint32_t *out)
{
	const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
	uint32_t acc = 0;
	for (size_t i = g; i < nvec; i += stride) {
		u32x4 v;
		asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p + i * 16) : "memory");
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x9e3779b9u)
		out[0] = acc;
}

__global__ __launch_bounds__(256) void rd_x1(const uint8_t *p, size_t nw, uint32_t *out)
{
	const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
	uint32_t acc = 0;
	for (size_t i = g; i < nw; i += stride) {
		uint32_t v;
		asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p + i * 4) : "memory");
		acc ^= v;
	}
	if (acc == 0x9e3779b9u)
		out[0] = acc;
}

int main()
{
	uint8_t *p;
	uint32_t *out;
	if (hipMalloc(&p, BYTES + 256) != hipSuccess || hipMalloc(&out, 64) != hipSuccess)
		return 1;
	(void)hipMemset(p, 1, BYTES + 256);
	(void)hipDeviceSynchronize();
	const int grid = 256 * 8 * 4;
	for (int r = 0; r < 3; r++) {
		rd_x4<<<grid, 256>>>(p, BYTES / 16, out);            // aligned 16 B/lane
		rd_x4<<<grid, 256>>>(p + 4, BYTES / 16, out);        // 4-B-aligned 16 B/lane
		rd_x1<<<grid, 256>>>(p, BYTES / 4, out);             // 4 B/lane
	}
	(void)hipDeviceSynchronize();
	printf("{\"bytes_per_launch\": %zu, \"order\": [\"x4 aligned\", \"x4 base+4\", \"x1\"], \"repeats\": 3}\n", BYTES);
	return 0;
}
