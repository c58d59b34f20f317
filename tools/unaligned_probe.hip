// Does gfx950 (under ROCm's SH_MEM_CONFIG) serve global_load_dword /
// global_load_dwordx4 at byte-aligned addresses with the bytes at those
// addresses (unaligned access mode), and at what cost?  One lane per
// packet, 64 KiB buffer of known bytes; every lane loads 4 x dwordx4 at
// base + lane*17 + off (off = 0..3) and compares with the byte pattern.
// Then a timing pass: 1 M lanes each read 128 B at a byte-aligned start
// through dwordx4 vs through aligned dwords + v_alignbyte (the kernels'
// A1 path), same XOR-reduction of the words.
//   hipcc --offload-arch=gfx950 -O3 tools/unaligned_probe.hip -o tools/unaligned_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gvec;
typedef __attribute__((address_space(1))) const uint32_t gword;

__global__ void check(const uint8_t *buf, uint32_t *bad)
{
	const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
	for (int off = 0; off < 4; off++) {
		const uint8_t *p = buf + lane * 17 + off;
		for (int k = 0; k < 4; k++) {
			u32x4 v = *(gvec *)(p + 16 * k);
			uint32_t w = *(gword *)(p + 16 * k + 4);
			for (int j = 0; j < 4; j++) {
				uint32_t want = 0;
				for (int b = 0; b < 4; b++)
					want |= (uint32_t)(uint8_t)((lane * 17 + off + 16 * k + 4 * j + b) * 7 + 3) << (8 * b);
				if (v[j] != want)
					atomicAdd(bad, 1u);
				if (j == 1 && w != want)
					atomicAdd(bad + 1, 1u);
			}
		}
	}
}

__global__ void time_x4(const uint8_t *buf, uint32_t *out, int off)
{
	const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
	const uint8_t *p = buf + (size_t)lane * 128 + off;
	uint32_t acc = 0;
#pragma unroll
	for (int k = 0; k < 8; k++) {
		u32x4 v = *(gvec *)(p + 16 * k);
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	out[lane] = acc;
}

__global__ void time_align(const uint8_t *buf, uint32_t *out, int off)
{
	const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
	const uintptr_t a = (uintptr_t)(buf + (size_t)lane * 128 + off);
	const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
	const uint32_t sh = (uint32_t)(a & 3) * 8;
	uint32_t d[33];
#pragma unroll
	for (int k = 0; k < 33; k++)
		d[k] = ((gword *)q)[k];
	uint32_t acc = 0;
#pragma unroll
	for (int k = 0; k < 32; k++)
		acc ^= __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh / 8);
	out[lane] = acc;
}

int main()
{
	const size_t n = 1 << 20, bytes = n * 128 + 256;
	uint8_t *h = (uint8_t *)malloc(bytes), *d;
	for (size_t i = 0; i < bytes; i++)
		h[i] = (uint8_t)(i * 7 + 3);
	uint32_t *bad, *out, hb[2];
	hipMalloc(&d, bytes);
	hipMalloc(&bad, 8);
	hipMalloc(&out, n * 4);
	hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
	hipMemset(bad, 0, 8);
	check<<<16, 256>>>(d, bad);
	hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost);
	printf("{\"unaligned_dwordx4_mismatches\": %u, \"unaligned_dword_mismatches\": %u", hb[0], hb[1]);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	for (int off = 0; off < 2; off++) {
		float best[2] = { 1e9f, 1e9f };
		for (int r = 0; r < 20; r++) {
			for (int v = 0; v < 2; v++) {
				hipEventRecord(e0);
				if (v == 0)
					time_x4<<<n / 256, 256>>>(d, out, off);
				else
					time_align<<<n / 256, 256>>>(d, out, off);
				hipEventRecord(e1);
				hipEventSynchronize(e1);
				float ms;
				hipEventElapsedTime(&ms, e0, e1);
				if (ms < best[v])
					best[v] = ms;
			}
		}
		printf(", \"off%d_x4_us\": %.1f, \"off%d_alignbyte_us\": %.1f", off,
		    best[0] * 1e3, off, best[1] * 1e3);
	}
	printf("}\n");
	return hb[0] || hb[1] ? 1 : 0;
}
