// kernel_ab.hip -- launch-shape A/B of the shipped SHA-256 fixed kernel body
// on the config-2 workload (1M x 1 KiB, device-resident).  All variants run
// the same lane code (fixed_lane from sha2_kernels.hip); only block size,
// register attributes and grid shape differ.  Outputs are compared.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ilias_net2_amd/csrc tools/kernel_ab.hip -o tools/kernel_ab
#define NET2_SHA2_NO_LAUNCHERS
#include "../ilias_net2_amd/csrc/sha2_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <functional>

using namespace net2::dev;
typedef PadKW<uint32_t> KW;

template <int BS>
__global__ __launch_bounds__(BS) void k_plain(const uint8_t *base, uint32_t len,
    uint64_t n, uint8_t *out, KW pad)
{
	const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
	if (i < n)
		fixed_lane<Sha256, AMODE_A16, true>(i, base, len, len, out, 32, 0, pad.kw);
}

/* the A4 / A1 load paths on the same (16-byte aligned) packets */
template <int AM>
__global__ __launch_bounds__(256) void k_amode(const uint8_t *base, uint32_t len,
    uint64_t n, uint8_t *out, KW pad)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	if (i < n)
		fixed_lane<Sha256, AM, true>(i, base, len, len, out, 32, 0, pad.kw);
}

template <int BS>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_num_sgpr(80)))
void k_sgpr80(const uint8_t *base, uint32_t len, uint64_t n, uint8_t *out, KW pad)
{
	const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
	if (i < n)
		fixed_lane<Sha256, AMODE_A16, true>(i, base, len, len, out, 32, 0, pad.kw);
}

/* grid-stride: gridDim.x blocks loop over the packets */
template <int BS>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_num_sgpr(80)))
void k_stride(const uint8_t *base, uint32_t len, uint64_t n, uint8_t *out, KW pad)
{
	for (uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x; i < n;
	    i += (uint64_t)gridDim.x * BS)
		fixed_lane<Sha256, AMODE_A16, true>(i, base, len, len, out, 32, 0, pad.kw);
}

/*
 * LDS-staged variant (the north-star's "blocks coalesced from HBM into an
 * LDS-staged schedule"): each wave owns a 4 KiB LDS slab holding block k of
 * its 64 packets.  Block k+1 is fetched with 4 global_load_lds_dwordx4 per
 * wave -- 16 packets x 64 B per instruction, 4 lanes per packet, so each
 * instruction touches 16 whole 64-B segments instead of 64 scattered
 * 16-B pieces -- while block k (already copied LDS -> VGPR) is compressed.
 * The LDS image is lane-linear; the chunk order inside a packet is XOR-
 * swizzled on the global side (c ^ (p>>2 & 3)) so that the per-lane
 * ds_read_b128 of a 64-B row is bank-conflict free.  Requires n % 64 == 0,
 * stride % 16 == 0, len % 64 == 0.
 */
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

__global__ __launch_bounds__(256) void k_lds(const uint8_t *base, uint32_t len,
    uint64_t n, uint8_t *out, KW pad)
{
	__shared__ u32x4 slab[4][256];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const uint64_t w0 = (uint64_t)blockIdx.x * 256 + wv * 64;
	const uint32_t nfull = len / 64;
	u32x4 *my = slab[wv];

	/* loader geometry: instruction j, lane l -> packet 16j + l/4 */
	auto issue = [&](uint32_t k) {
#pragma unroll
		for (int j = 0; j < 4; j++) {
			const int p = 16 * j + (lane >> 2);
			const int c = (lane & 3) ^ ((p >> 2) & 3);
			const uint8_t *g = base + (w0 + p) * (uint64_t)len + k * 64 + c * 16;
			__builtin_amdgcn_global_load_lds((glb_void *)g,
			    (lds_void *)(my + 64 * j), 16, 0, 0);
		}
	};
	uint32_t st[8];
	Sha256::init(st, 0);
	issue(0);
	const int f = (lane >> 2) & 3;
	for (uint32_t k = 0; k < nfull; k++) {
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		uint32_t w[16];
#pragma unroll
		for (int c = 0; c < 4; c++) {
			u32x4 v = my[4 * lane + (c ^ f)];
			w[4 * c] = bswap32(v.x);
			w[4 * c + 1] = bswap32(v.y);
			w[4 * c + 2] = bswap32(v.z);
			w[4 * c + 3] = bswap32(v.w);
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		if (k + 1 < nfull)
			issue(k + 1);
		compress256(st, w);
	}
	compress256_kw(st, pad.kw);
	uint32_t o[16];
	Sha256::out_words(st, o, 0);
	store_digest<32>(out + (w0 + lane) * 32, o);
}

typedef PadKW<uint64_t> KW5;

template <int AM, bool PF>
__global__ __launch_bounds__(256) void k512(const uint8_t *base, uint32_t len,
    uint64_t n, uint8_t *out, KW5 pad)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	k512_lds_fill_pad(pad);
	if (i < n)
		fixed_lane<Sha512, AM, true, PF>(i, base, len, len, out, 64, 0, pad.kw);
}

#define K512V(V)                                                                 \
	__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(V)))    \
	void k512v##V(const uint8_t *base, uint32_t len, uint64_t n, uint8_t *out, KW5 pad) \
	{                                                                        \
		const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;     \
		k512_lds_fill_pad(pad);                                           \
		if (i < n)                                                       \
			fixed_lane<Sha512, AMODE_A16, true, false>(i, base, len, len, out, 64, 0, pad.kw); \
	}
K512V(96)
K512V(80)
K512V(64)

template <class F>
static float best_of(F launch, int reps)
{
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	float best = 1e9;
	for (int r = 0; r < reps; r++) {
		(void)hipEventRecord(a);
		launch();
		(void)hipEventRecord(b);
		(void)hipEventSynchronize(b);
		float ms;
		(void)hipEventElapsedTime(&ms, a, b);
		best = std::min(best, ms);
	}
	return best;
}

int main()
{
	const uint64_t n = 1 << 20;
	const uint32_t len = 1024;
	uint8_t *d_in, *d_out;
	(void)hipMalloc(&d_in, n * len);
	(void)hipMalloc(&d_out, n * 64 * 8);
	std::vector<uint8_t> h(n * len);
	uint64_t x = 88172645463325252ull;
	for (size_t i = 0; i < h.size(); i += 8) {
		x ^= x << 13; x ^= x >> 7; x ^= x << 17;
		memcpy(&h[i], &x, 8);
	}
	(void)hipMemcpy(d_in, h.data(), h.size(), hipMemcpyHostToDevice);
	KW pad;
	pad_kw256((uint64_t)len << 3, pad);
	KW5 pad5;
	pad_kw512((uint64_t)len << 3, pad5);
	const bool do512 = getenv("AB512") != nullptr;

	hipDeviceProp_t p;
	(void)hipGetDeviceProperties(&p, 0);
	const int cus = p.multiProcessorCount;
	struct V { const char *name; std::function<void(uint8_t *)> f; };
	std::vector<V> vs512 = {
		{"S0 sha512 A16 no-prefetch (shipped)", [&](uint8_t *o) { k512<AMODE_A16, false><<<n / 256, 256>>>(d_in, len, n, o, pad5); }},
		{"S1 sha512 A16 prefetch", [&](uint8_t *o) { k512<AMODE_A16, true><<<n / 256, 256>>>(d_in, len, n, o, pad5); }},
		{"S2 sha512 A1 path", [&](uint8_t *o) { k512<AMODE_A1, false><<<n / 256, 256>>>(d_in, len, n, o, pad5); }},
		{"S3 sha512 A16 vgpr<=96", [&](uint8_t *o) { k512v96<<<n / 256, 256>>>(d_in, len, n, o, pad5); }},
		{"S4 sha512 A16 vgpr<=80", [&](uint8_t *o) { k512v80<<<n / 256, 256>>>(d_in, len, n, o, pad5); }},
		{"S5 sha512 A16 vgpr<=64", [&](uint8_t *o) { k512v64<<<n / 256, 256>>>(d_in, len, n, o, pad5); }},
	};
	std::vector<V> vs = {
		{"A block256 (shipped)", [&](uint8_t *o) { k_plain<256><<<n / 256, 256>>>(d_in, len, n, o, pad); }},
		{"B block64", [&](uint8_t *o) { k_plain<64><<<n / 64, 64>>>(d_in, len, n, o, pad); }},
		{"C block128", [&](uint8_t *o) { k_plain<128><<<n / 128, 128>>>(d_in, len, n, o, pad); }},
		{"D block256 sgpr80", [&](uint8_t *o) { k_sgpr80<256><<<n / 256, 256>>>(d_in, len, n, o, pad); }},
		{"E block64 sgpr80", [&](uint8_t *o) { k_sgpr80<64><<<n / 64, 64>>>(d_in, len, n, o, pad); }},
		{"F stride 256x(8/CU) sgpr80", [&](uint8_t *o) { k_stride<256><<<cus * 8, 256>>>(d_in, len, n, o, pad); }},
		{"G stride 64x(32/CU) sgpr80", [&](uint8_t *o) { k_stride<64><<<cus * 32, 64>>>(d_in, len, n, o, pad); }},
		{"H block256 A4 (dword loads)", [&](uint8_t *o) { k_amode<AMODE_A4><<<n / 256, 256>>>(d_in, len, n, o, pad); }},
		{"I block256 A1 (dword + alignbyte)", [&](uint8_t *o) { k_amode<AMODE_A1><<<n / 256, 256>>>(d_in, len, n, o, pad); }},
		{"L block256 LDS-staged glds", [&](uint8_t *o) { k_lds<<<n / 256, 256>>>(d_in, len, n, o, pad); }},
	};
	if (do512)
		vs = vs512;
	const int DL = do512 ? 64 : 32;
	std::vector<float> best(vs.size(), 1e9);
	for (size_t v = 0; v < vs.size(); v++)
		vs[v].f(d_out + v * n * DL);  // warm-up
	(void)hipDeviceSynchronize();
	for (int round = 0; round < 4; round++)
		for (size_t v = 0; v < vs.size(); v++)
			best[v] = std::min(best[v], best_of([&] { vs[v].f(d_out + v * n * DL); }, 3));
	std::vector<uint8_t> ref(n * DL), got(n * DL);
	(void)hipMemcpy(ref.data(), d_out, n * DL, hipMemcpyDeviceToHost);
	printf("{\"n\": %llu, \"len\": %u, \"variants\": [\n", (unsigned long long)n, len);
	for (size_t v = 0; v < vs.size(); v++) {
		(void)hipMemcpy(got.data(), d_out + v * n * DL, n * DL, hipMemcpyDeviceToHost);
		printf("  {\"variant\": \"%s\", \"ms\": %.4f, \"Gdigests_per_s\": %.4f, \"same\": %s}%s\n",
		    vs[v].name, best[v], n / (best[v] * 1e-3) / 1e9,
		    got == ref ? "true" : "false", v + 1 == vs.size() ? "" : ",");
	}
	printf("]}\n");
	return 0;
}
