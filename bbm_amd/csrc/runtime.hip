// bbm_amd/csrc/runtime.hip -- the host-side pieces of the fitting path that sit around the loss kernels:
//
//   * bbm_hip_rng_*: bbm::rng<Size_t> (backbone/native/include/backbone/random.h:40-66), the generator behind
//     bbm::batch (include/bbm/batch.h:27-92) -- std::mt19937_64 and libstdc++'s uniform_int_distribution, restated
//     so that a batch drawn here holds the reference's indices for the same seed;
//   * bbm_hip_gather_samples(_f64): a batch's samples gathered densely from the materialised pairs / reference
//     table (one device pass), ready for any loss entry point;
//   * bbm_hip_comm_* / bbm_hip_allreduce_sums: an RCCL communicator for the loss reduction of a sharded fit (the
//     2P probe sums of a compass step, include/optimizer/compass.h:122), RCCL loaded at run time.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bbm_hip.h"

namespace bbmhip {
int fail(int code, const std::string& msg);
std::string scratch_failure();
void* scratch_acquire(size_t bytes, hipStream_t s);
void scratch_release(void* p, hipStream_t s);
}  // namespace bbmhip

using namespace bbmhip;

namespace {

// ------------------------------------------------------------------------------------------ mt19937_64
// The standard's parameters ([rand.predef]: mersenne_twister_engine<uint_fast64_t, 64, 312, 156, 31,
// 0xb5026f5aa96619e9, 29, 0x5555555555555555, 17, 0x71d67fffeda60000, 37, 0xfff7eee000000000, 43,
// 6364136223846793005>), state refilled in one pass as libstdc++'s _M_gen_rand does.
constexpr int kN = 312, kM = 156;
constexpr uint64_t kMatrixA = 0xb5026f5aa96619e9ull;
constexpr uint64_t kUpper = ~uint64_t(0) << 31, kLower = ~kUpper;

void mt_seed(bbm_hip_rng* r, uint64_t seed)
{
  r->mt[0] = seed;
  for (int i = 1; i < kN; ++i) r->mt[i] = 6364136223846793005ull * (r->mt[i - 1] ^ (r->mt[i - 1] >> 62)) + uint64_t(i);
  r->pos = kN;
}

void mt_refill(bbm_hip_rng* r)
{
  uint64_t* mt = r->mt;
  for (int k = 0; k < kN - kM; ++k)
  {
    const uint64_t y = (mt[k] & kUpper) | (mt[k + 1] & kLower);
    mt[k] = mt[k + kM] ^ (y >> 1) ^ ((y & 1) ? kMatrixA : 0);
  }
  for (int k = kN - kM; k < kN - 1; ++k)
  {
    const uint64_t y = (mt[k] & kUpper) | (mt[k + 1] & kLower);
    mt[k] = mt[k + (kM - kN)] ^ (y >> 1) ^ ((y & 1) ? kMatrixA : 0);
  }
  const uint64_t y = (mt[kN - 1] & kUpper) | (mt[0] & kLower);
  mt[kN - 1] = mt[kM - 1] ^ (y >> 1) ^ ((y & 1) ? kMatrixA : 0);
  r->pos = 0;
}

uint64_t mt_next(bbm_hip_rng* r)
{
  if (r->pos >= kN) mt_refill(r);
  uint64_t z = r->mt[r->pos++];
  z ^= (z >> 29) & 0x5555555555555555ull;
  z ^= (z << 17) & 0x71d67fffeda60000ull;
  z ^= (z << 37) & 0xfff7eee000000000ull;
  z ^= z >> 43;
  return z;
}

// libstdc++ 11 uniform_int_distribution<uint64_t>::operator() (bits/uniform_int_dist.h): the generator's range is the
// full 64 bits, so [a, b] is drawn by Lemire's nearly divisionless method (_S_nd) in 128-bit arithmetic on b - a + 1
// values; b - a + 1 == 0 (the full range) returns the generator's output itself.
uint64_t uniform(bbm_hip_rng* r)
{
  const uint64_t range = r->upper - r->lower + 1;
  if (range == 0) return r->lower + mt_next(r);
  unsigned __int128 product = (unsigned __int128)mt_next(r) * range;
  uint64_t low = uint64_t(product);
  if (low < range)
  {
    const uint64_t threshold = (0 - range) % range;
    while (low < threshold)
    {
      product = (unsigned __int128)mt_next(r) * range;
      low = uint64_t(product);
    }
  }
  return r->lower + uint64_t(product >> 64);
}

// ------------------------------------------------------------------------------------------ gather
constexpr int kMaxGather = 16;
template<class T> struct GatherArgs { const T* src[kMaxGather]; T* dst[kMaxGather]; };

template<class T>
__global__ __launch_bounds__(256) void k_gather(GatherArgs<T> a, int narrays, const uint64_t* index, uint64_t n)
{
  const uint64_t stride = uint64_t(gridDim.x) * 256;
  for (uint64_t j = uint64_t(blockIdx.x) * 256 + threadIdx.x; j < n; j += stride)
  {
    const uint64_t i = index[j];
    for (int k = 0; k < narrays; ++k) a.dst[k][j] = a.src[k][i];
  }
}

template<class T>
int gather(const uint64_t* index, size_t count, uint64_t nsamples, const T* const* src, T* const* dst, int narrays,
           void* stream)
{
  if (narrays < 1 || narrays > kMaxGather) return fail(BBM_HIP_ERR_INVALID_ARG, "narrays must be in [1, 16]");
  if (count > 0 && !index) return fail(BBM_HIP_ERR_INVALID_ARG, "index is NULL");
  if (!src || !dst) return fail(BBM_HIP_ERR_INVALID_ARG, "src / dst is NULL");
  GatherArgs<T> a{};
  for (int k = 0; k < narrays; ++k)
  {
    if (!src[k] || !dst[k]) return fail(BBM_HIP_ERR_INVALID_ARG, "array pointer is NULL");
    a.src[k] = src[k];
    a.dst[k] = dst[k];
  }
  // the batch's samples in draw order; an index past the last sample is the reference's masked lane
  // (sampledlossfunction.h:65-66 returns 0 for it) and is left out
  std::vector<uint64_t> keep;
  keep.reserve(count);
  for (size_t j = 0; j < count; ++j)
    if (index[j] < nsamples) keep.push_back(index[j]);
  if (keep.empty()) return 0;
  if (keep.size() > size_t(INT32_MAX)) return fail(BBM_HIP_ERR_INVALID_ARG, "batch too large");
  const hipStream_t s = static_cast<hipStream_t>(stream);
  void* di = scratch_acquire(keep.size() * sizeof(uint64_t), s);
  if (!di) return fail(BBM_HIP_ERR_HIP, "gather indices: scratch allocation failed: " + scratch_failure());
  hipError_t e = hipMemcpyAsync(di, keep.data(), keep.size() * sizeof(uint64_t), hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
  {
    uint64_t blocks = (keep.size() + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL((k_gather<T>), dim3(unsigned(blocks)), dim3(256), 0, s, a, narrays,
                       static_cast<const uint64_t*>(di), uint64_t(keep.size()));
    e = hipGetLastError();
  }
  // the host vector is staged by the copy before the stream runs on: wait for it before `keep` goes away
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  scratch_release(di, s);
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("gather: ") + hipGetErrorString(e));
  return int(keep.size());
}

// ------------------------------------------------------------------------------------------ RCCL
// librccl is opened on first use (the process may already hold torch's copy: dlopen then returns that one), so the
// library does not depend on RCCL unless a communicator is made.
struct Rccl
{
  bool ok = false;
  std::string why;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl()
{
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h)
    {
      const char* e = dlerror();
      r.why = std::string("cannot load librccl: ") + (e ? e : "unknown error");
      return;
    }
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.init_rank && r.destroy && r.all_reduce && r.error_string;
    if (!r.ok) r.why = "librccl lacks an NCCL entry point";
  });
  return r;
}

int rccl_fail(const Rccl& r, ncclResult_t e, const char* what)
{
  return fail(BBM_HIP_ERR_HIP, std::string(what) + ": " + (r.error_string ? r.error_string(e) : "RCCL error"));
}

}  // namespace

struct bbm_hip_comm
{
  ncclComm_t comm;
  int rank, world, device;
};

extern "C" {

int bbm_hip_rng_init(bbm_hip_rng* rng, uint64_t seed, uint64_t lower, uint64_t upper)
{
  if (!rng) return fail(BBM_HIP_ERR_INVALID_ARG, "rng is NULL");
  if (upper < lower) return fail(BBM_HIP_ERR_INVALID_ARG, "rng: upper < lower");
  mt_seed(rng, seed);
  rng->lower = lower;
  rng->upper = upper;
  rng->magic = BBM_HIP_RNG_MAGIC;
  return BBM_HIP_OK;
}

int bbm_hip_rng_draw(bbm_hip_rng* rng, uint64_t* out, size_t n)
{
  if (!rng || (n > 0 && !out)) return fail(BBM_HIP_ERR_INVALID_ARG, "rng / out is NULL");
  if (rng->magic != BBM_HIP_RNG_MAGIC || rng->pos > uint64_t(kN) || rng->upper < rng->lower)
    return fail(BBM_HIP_ERR_INVALID_ARG, "rng not initialised (bbm_hip_rng_init)");
  for (size_t i = 0; i < n; ++i) out[i] = uniform(rng);
  return BBM_HIP_OK;
}

int bbm_hip_gather_samples(const uint64_t* index, size_t count, uint64_t nsamples, const float* const* src,
                           float* const* dst, int narrays, void* stream)
{
  return gather<float>(index, count, nsamples, src, dst, narrays, stream);
}

int bbm_hip_gather_samples_f64(const uint64_t* index, size_t count, uint64_t nsamples, const double* const* src,
                               double* const* dst, int narrays, void* stream)
{
  return gather<double>(index, count, nsamples, src, dst, narrays, stream);
}

int bbm_hip_comm_unique_id(uint8_t* id, size_t bytes)
{
  if (!id || bytes != BBM_HIP_COMM_ID_BYTES) return fail(BBM_HIP_ERR_INVALID_ARG, "id must hold BBM_HIP_COMM_ID_BYTES bytes");
  static_assert(sizeof(ncclUniqueId) == BBM_HIP_COMM_ID_BYTES, "RCCL unique id size");
  const Rccl& r = rccl();
  if (!r.ok) return fail(BBM_HIP_ERR_UNSUPPORTED, r.why);
  ncclUniqueId u;
  const ncclResult_t e = r.get_unique_id(&u);
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof(u));
  return BBM_HIP_OK;
}

int bbm_hip_comm_init(const uint8_t* id, size_t bytes, int rank, int world, bbm_hip_comm** comm)
{
  if (!comm) return fail(BBM_HIP_ERR_INVALID_ARG, "comm is NULL");
  *comm = nullptr;
  if (!id || bytes != BBM_HIP_COMM_ID_BYTES) return fail(BBM_HIP_ERR_INVALID_ARG, "id must hold BBM_HIP_COMM_ID_BYTES bytes");
  if (world < 1 || rank < 0 || rank >= world) return fail(BBM_HIP_ERR_INVALID_ARG, "rank / world out of range");
  const Rccl& r = rccl();
  if (!r.ok) return fail(BBM_HIP_ERR_UNSUPPORTED, r.why);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(BBM_HIP_ERR_HIP, "no current HIP device");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const ncclResult_t e = r.init_rank(&c, world, u, rank);
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommInitRank");
  *comm = new bbm_hip_comm{c, rank, world, dev};
  return BBM_HIP_OK;
}

int bbm_hip_comm_destroy(bbm_hip_comm* comm)
{
  if (!comm) return BBM_HIP_OK;
  const Rccl& r = rccl();
  const ncclResult_t e = r.destroy(comm->comm);
  delete comm;
  return e == ncclSuccess ? BBM_HIP_OK : rccl_fail(r, e, "ncclCommDestroy");
}

int bbm_hip_comm_rank(const bbm_hip_comm* comm)
{
  return comm ? comm->rank : fail(BBM_HIP_ERR_INVALID_ARG, "comm is NULL");
}

int bbm_hip_comm_size(const bbm_hip_comm* comm)
{
  return comm ? comm->world : fail(BBM_HIP_ERR_INVALID_ARG, "comm is NULL");
}

int bbm_hip_allreduce_sums(bbm_hip_comm* comm, double* sums, size_t n, void* stream)
{
  if (!comm) return fail(BBM_HIP_ERR_INVALID_ARG, "comm is NULL");
  if (n == 0) return BBM_HIP_OK;
  if (!sums) return fail(BBM_HIP_ERR_INVALID_ARG, "sums is NULL");
  const Rccl& r = rccl();
  const ncclResult_t e = r.all_reduce(sums, sums, n, ncclFloat64, ncclSum, comm->comm, static_cast<hipStream_t>(stream));
  return e == ncclSuccess ? BBM_HIP_OK : rccl_fail(r, e, "ncclAllReduce");
}

}  // extern "C"
