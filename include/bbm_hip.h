/* include/bbm_hip.h -- C-ABI of libbbm_hip.so, the MI355X (gfx950) batched BSDF backbone.
 *
 * This is the drop-in boundary for BBM's hot path.  In the reference, a bsdfmodel<> is evaluated
 * one (in, out) pair per call through the template API of the bsdfmodel concept
 * (include/concepts/bsdfmodel.h:33-146):
 *
 *   Spectrum   eval(const Vec3d& in, const Vec3d& out, BsdfFlag component, unit_t unit, Mask mask)
 *   Value      pdf(const Vec3d& in, const Vec3d& out, BsdfFlag component, unit_t unit, Mask mask)
 *   BsdfSample sample(const Vec3d& out, const Vec2d& xi, BsdfFlag component, unit_t unit, Mask mask)
 *   Spectrum   reflectance(const Vec3d& out, BsdfFlag component, unit_t unit, Mask mask)
 *
 * and batching only exists when the backbone's Value is a wide type (backbone/enoki,
 * backbone/drjit).  Here the same four calls take N pairs at once: directions are SoA float32
 * device arrays (x[], y[], z[]), the per-lane Mask is an optional uint8 array, and `component` /
 * `unit` are uniform per call.  Model parameters are the flat bbm::parameter_values() vector
 * (include/bbm/bsdf_enumerate.h; attribute declaration order, Dependent attributes included),
 * uniform per call.  All pointers are caller-owned device memory; calls are asynchronous on
 * `stream` (a hipStream_t; NULL = the default stream) and never synchronise.
 *
 * Errors: the reference throws C++ exceptions (include/core/error.h:42-46); here every entry
 * point returns BBM_HIP_OK (0) or a negative code and records a message readable through
 * bbm_hip_last_error() (thread-local).  No exception crosses this ABI.
 */
#ifndef BBM_HIP_H
#define BBM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BBM_HIP_ABI_VERSION 12

/* return codes */
#define BBM_HIP_OK 0
#define BBM_HIP_ERR_INVALID_MODEL -1   /* unknown model id / name (reference: std::invalid_argument, bsdf_string_convert.h:70-75) */
#define BBM_HIP_ERR_INVALID_ARG -2     /* null pointer, bad parameter count, ... */
#define BBM_HIP_ERR_UNSUPPORTED -3     /* operation not (yet) available for this model */
#define BBM_HIP_ERR_HIP -4             /* HIP runtime error (launch failure) */

/* bsdf_flag (include/bbm/bsdf_flag.h:21-27) */
#define BBM_FLAG_NONE 0u
#define BBM_FLAG_DIFFUSE 1u
#define BBM_FLAG_SPECULAR 2u
#define BBM_FLAG_ALL 3u

/* unit_t (include/bbm/unit.h:20-24) */
#define BBM_UNIT_RADIANCE 0u
#define BBM_UNIT_IMPORTANCE 1u

/* ---------------------------------------------------------------- library / registry */

/* ABI version of the loaded library (BBM_HIP_ABI_VERSION). */
int bbm_hip_abi_version(void);

/* Last error message of the calling thread ("" if none). */
const char* bbm_hip_last_error(void);

/* Exact-subnormal mode (process-wide, default off; initial value from the environment variable
 * BBM_HIP_EXACT_SUBNORMALS).  On: the eval / pdf kernels of the Beckmann microfacet models (CookTorrance and its
 * Walter / Heitz / Ngan variants) take the three quotients a subnormal intermediate can reach (D, the Cook
 * normalisation, the pdf's 1 / (4 |o.h|)) with a double remainder step, so eval and pdf are the reference's floats
 * bit for bit on every lane (ndf/beckmann.h:60 -> glibc expf, microfacet.h:100, :171), at +3.6-4.3 % kernel time on
 * the headline.  Also Bagher's NDF (ndf/sgd.h:56-62: pow(temp, p) and exp(-temp) as glibc's own powf / expf instead
 * of ~1e-6 approximations; +68 % Bagher kernel time), the Low and Student-T NDFs' double pow (ndf/low.h:53,
 * ndf/studentt.h:53: LowMicrofacet(Fit), Ribardiere) computed in double and rounded to float, and every fused
 * Aggregate(Lambertian, X) whose X has an exact mode.  Sampling (bbm_hip_sample, bbm_hip_check's sampling tests):
 * the Beckmann visible-normal sampler starts its Newton steps from glibc's erff / logf (ndf/beckmann.h:94-96) and
 * GGX's takes glibc's sinf / cosf of its azimuth (ndf/ggx.h:99) instead of the device library's (+28 % / +7 % on
 * importance-sampled reflectance).  Off: those quotients use the f32 remainder step, Bagher's D the fast power and
 * the samplers the device functions; outputs may differ in the last bits (the per-lane parity bar holds either way).
 * Returns the previous setting (0 / 1), or a negative code.  The switch is the process-wide DEFAULT: a call whose
 * model id carries BBM_HIP_CALL_EXACT (or BBM_HIP_CALL_DEFAULT) runs in exact (or default) mode whatever the switch
 * says, so a caller that must not depend on another thread's setting passes one of the two bits (re-entrant: the
 * bit is decoded per call, on the calling thread).  The bits may be OR-ed into the id given to any entry point that
 * takes a model id (eval / pdf / eval_pdf / sample / reflectance, loss, check; a child's id in a tree applies to
 * that child); they are ignored by the doubleRGB kernels, which have no exact mode. */
int bbm_hip_set_exact_subnormals(int on);
#define BBM_HIP_CALL_EXACT 0x20000000
#define BBM_HIP_CALL_DEFAULT 0x10000000

/* Model registry.  Replaces the compile-time registry of BBM_EXPORT_BSDFMODEL
 * (e.g. include/bsdfmodel/cooktorrance.h:42) and the keyword lookup of
 * fromString<bsdf_ptr> (include/bbm/bsdf_string_convert.h:52-82). */
int bbm_hip_num_models(void);
const char* bbm_hip_model_name(int model_id);          /* NULL if out of range */
int bbm_hip_model_id(const char* name);                 /* <0 if unknown */
int bbm_hip_model_nparams(int model_id);                /* length of the parameter vector */
/* Default / lower / upper parameter vectors (bsdf_attribute.h defaults and bounds;
 * bbm::parameter_default_values / parameter_lower_bound / parameter_upper_bound,
 * include/bbm/bsdf_enumerate.h).  which: 0 = default, 1 = lower, 2 = upper.  Returns nparams. */
int bbm_hip_model_params(int model_id, int which, float* out, int capacity);
/* Component flags the model can return non-zero values for (BBM_FLAG_*). */
int bbm_hip_model_components(int model_id);
/* Per-parameter bsdf_attr flags (include/bbm/bsdf_attr_flag.h:16-29: DiffuseScale 0x01,
 * DiffuseParameter 0x02, SpecularScale 0x04, SpecularParameter 0x08, Dependent 0x10), i.e. which
 * entries bbm::parameter_values(model, flag) selects (include/bbm/bsdf_enumerate.h:103-131; the
 * default flag All = 0x0F leaves out Dependent attributes).  Returns nparams. */
int bbm_hip_model_param_attrs(int model_id, uint32_t* out, int capacity);

/* ---------------------------------------------------------------- batched evaluation */

/* eval (RGB Spectrum) for n pairs -- bsdfmodel::eval, e.g. bsdfmodel/microfacet.h:74-102. */
int bbm_hip_eval(int model_id, const float* params, int nparams,
                 const float* in_x, const float* in_y, const float* in_z,
                 const float* out_x, const float* out_y, const float* out_z,
                 const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                 float* r, float* g, float* b, void* stream);

/* pdf for n pairs -- bsdfmodel::pdf, e.g. bsdfmodel/microfacet.h:154-174. */
int bbm_hip_pdf(int model_id, const float* params, int nparams,
                const float* in_x, const float* in_y, const float* in_z,
                const float* out_x, const float* out_y, const float* out_z,
                const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                float* pdf, void* stream);

/* Fused eval + pdf over the same pairs (one read of the directions, one kernel): the headline
 * path (BASELINE.json metric).  Results are identical to bbm_hip_eval + bbm_hip_pdf. */
int bbm_hip_eval_pdf(int model_id, const float* params, int nparams,
                     const float* in_x, const float* in_y, const float* in_z,
                     const float* out_x, const float* out_y, const float* out_z,
                     const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                     float* r, float* g, float* b, float* pdf, void* stream);

/* sample (direction, pdf, flag) for n (out, xi) -- bsdfmodel::sample, e.g. microfacet.h:115-141.
 * flag receives the bsdf_flag of each sample (BBM_FLAG_*). */
int bbm_hip_sample(int model_id, const float* params, int nparams,
                   const float* out_x, const float* out_y, const float* out_z,
                   const float* xi0, const float* xi1,
                   const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                   float* dir_x, float* dir_y, float* dir_z, float* pdf, uint32_t* flag,
                   void* stream);

/* reflectance (RGB) for n outgoing directions -- bsdfmodel::reflectance, the (approximate)
 * hemispherical reflectance, e.g. bsdfmodel/microfacet.h:182-196, lambertian.h:136-140; the
 * weights aggregatemodel uses to mix its children's pdfs (aggregatemodel.h:81-150). */
int bbm_hip_reflectance(int model_id, const float* params, int nparams,
                        const float* out_x, const float* out_y, const float* out_z,
                        const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                        float* r, float* g, float* b, void* stream);

/* ---------------------------------------------------------------- doubleRGB (Value = double) */

/* The reference's doubleRGB configuration (backbone/native/include/backbone.h:41-42: Value = double, Spectrum =
 * color<double>): the same calls on SoA float64 arrays with a double parameter vector, evaluated in f64 on the
 * device.  Available for the models bbm_hip_model_has_f64 reports (every analytic model and their Aggregate(Lambertian, X) fits); BBM_HIP_ERR_UNSUPPORTED for the others. */
int bbm_hip_model_has_f64(int model_id);                /* 1 / 0, <0 for an unknown id */
int bbm_hip_eval_pdf_f64(int model_id, const double* params, int nparams,
                         const double* in_x, const double* in_y, const double* in_z,
                         const double* out_x, const double* out_y, const double* out_z,
                         const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                         double* r, double* g, double* b, double* pdf, void* stream);
int bbm_hip_sample_f64(int model_id, const double* params, int nparams,
                       const double* out_x, const double* out_y, const double* out_z,
                       const double* xi0, const double* xi1,
                       const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                       double* dir_x, double* dir_y, double* dir_z, double* pdf, uint32_t* flag, void* stream);
int bbm_hip_reflectance_f64(int model_id, const double* params, int nparams,
                            const double* out_x, const double* out_y, const double* out_z,
                            const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                            double* r, double* g, double* b, void* stream);

/* ---------------------------------------------------------------- aggregates of any models */

/* aggregatemodel<MODELS...> (include/bsdfmodel/aggregatemodel.h:22-222) of any >= 2 models, each child given as
 * (model id, its parameter vector): replaces the reference's variadic template instantiation (aggregatemodel.h:222
 * `aggregatemodel<MODELS...>`, aggregate() :232-233) for compositions that have no fused registry entry
 * ("Aggregate<Lambertian,X>").  A child may itself be a composed aggregate (the reference's aggregatemodel_base
 * takes any bsdfmodel child, :22, including another aggregate): model_id = BBM_HIP_AGGREGATE, params unused, and
 * its own children in `children` / `nchildren` (any depth).  Evaluated by composing the children's kernels (one
 * pass per child; eval and reflectance as the reference's right fold, pdf as the reflectance-weighted mixture,
 * sample by the reference's child selection on xi0, each nested aggregate exactly as its own aggregatemodel
 * member functions would).  Same conventions as the single-model entry points; `r` may be NULL in
 * bbm_hip_aggregate_eval_pdf for pdf only, `pdf` NULL for eval only. */
#define BBM_HIP_AGGREGATE (-100)
/* The reference's RUNTIME aggregate, aggregatebsdf (include/bbm/aggregatebsdf.h:40-190): what fromString<bsdf_ptr> /
 * bsdf_import builds from "Aggregate(...)" (bsdf_string_convert.h:59), i.e. what checkBsdf, plotBsdf and the
 * Mitsuba plugin evaluate.  It differs from aggregatemodel in rounding and in one behaviour: eval and reflectance
 * are LEFT folds from 0, the pdf adds w_k pdf_k / sum term by term, and sample returns no sample (here {0, 0, None};
 * the reference's is indeterminate) unless sum > eps.  As a node kind in a child tree; as a flag OR-ed into the model
 * id of a fused Aggregate<A,B> entry (bbm_hip_eval / _pdf / _eval_pdf / _sample / _reflectance / _check and their
 * _f64 forms), the fused kernel takes these semantics.  bbm_hip_parse_model(_tree) returns both for strings. */
#define BBM_HIP_AGGREGATE_BSDF (-101)
#define BBM_HIP_RUNTIME_AGGREGATE 0x40000000
/* A tree may also be passed as its root alone: nchildren = 1 and children[0] an aggregate node (BBM_HIP_AGGREGATE
 * or BBM_HIP_AGGREGATE_BSDF) -- the only way to give the top level aggregatebsdf semantics. */
typedef struct bbm_hip_child
{
  int model_id;                            /* registry id (may carry BBM_HIP_RUNTIME_AGGREGATE), or an aggregate node */
  const float* params;                     /* host memory, nparams floats (bbm_hip_model_nparams); aggregate: NULL */
  int nparams;                             /* aggregate: 0 */
  const struct bbm_hip_child* children;    /* aggregate node: its children; else NULL */
  int nchildren;                           /* aggregate node: >= 2; else 0 */
} bbm_hip_child;

int bbm_hip_aggregate_eval_pdf(const bbm_hip_child* children, int nchildren,
                               const float* in_x, const float* in_y, const float* in_z,
                               const float* out_x, const float* out_y, const float* out_z,
                               const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                               float* r, float* g, float* b, float* pdf, void* stream);
int bbm_hip_aggregate_sample(const bbm_hip_child* children, int nchildren,
                             const float* out_x, const float* out_y, const float* out_z,
                             const float* xi0, const float* xi1,
                             const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                             float* dir_x, float* dir_y, float* dir_z, float* pdf, uint32_t* flag, void* stream);
int bbm_hip_aggregate_reflectance(const bbm_hip_child* children, int nchildren,
                                  const float* out_x, const float* out_y, const float* out_z,
                                  const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                                  float* r, float* g, float* b, void* stream);

/* The same in doubleRGB (Value = double): every leaf must have doubleRGB kernels (bbm_hip_model_has_f64); the
 * combining arithmetic (folds, weights, mixture, child selection) is the reference's in double. */
typedef struct bbm_hip_child_f64
{
  int model_id;
  const double* params;
  int nparams;
  const struct bbm_hip_child_f64* children;
  int nchildren;
} bbm_hip_child_f64;

int bbm_hip_aggregate_eval_pdf_f64(const bbm_hip_child_f64* children, int nchildren,
                                   const double* in_x, const double* in_y, const double* in_z,
                                   const double* out_x, const double* out_y, const double* out_z,
                                   const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                                   double* r, double* g, double* b, double* pdf, void* stream);
int bbm_hip_aggregate_sample_f64(const bbm_hip_child_f64* children, int nchildren,
                                 const double* out_x, const double* out_y, const double* out_z,
                                 const double* xi0, const double* xi1,
                                 const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                                 double* dir_x, double* dir_y, double* dir_z, double* pdf, uint32_t* flag,
                                 void* stream);
int bbm_hip_aggregate_reflectance_f64(const bbm_hip_child_f64* children, int nchildren,
                                      const double* out_x, const double* out_y, const double* out_z,
                                      const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                                      double* r, double* g, double* b, void* stream);

/* ---------------------------------------------------------------- model strings */

/* Attribute layout of a single model, "name:count,..." in declaration order (the order of its parameter
 * vector and of toString); NULL for aggregates / unknown ids. */
const char* bbm_hip_model_layout(int model_id);

/* Parse a model string -- bbm::toString form, an entry of the fits/ files, `Aggregate(child, child, ...)` -- as the
 * reference's runtime fromString does (include/bbm/bsdf_string_convert.h:52-85; the handle behind bsdf_ptr,
 * checkBsdf and the Mitsuba plugin).  A single model or an aggregate with a fused kernel yields ONE entry
 * (model_ids[0], its nparams[0] parameters; a fused aggregate's id carries BBM_HIP_RUNTIME_AGGREGATE); any other
 * aggregate yields one entry per child, to be evaluated with bbm_hip_aggregate_* as the children of a
 * BBM_HIP_AGGREGATE_BSDF root node (a child may be a fused aggregate).  Parameters are written back to back into params.
 * Returns the number of entries (>= 1) or an error code (unknown model / attribute, malformed string, value beyond
 * the float range; BBM_HIP_ERR_UNSUPPORTED for a composed aggregate nested inside another: use
 * bbm_hip_parse_model_tree). */
int bbm_hip_parse_model(const char* str, int* model_ids, float* params, int* nparams, int max_children,
                        int params_capacity);

/* The same for any nesting, as a tree in preorder: node k is model_ids[k] (a registry id, or BBM_HIP_AGGREGATE_BSDF
 * for a composed aggregate, whose nchildren[k] >= 2 children follow it in preorder; 0 for a registry model) with
 * nparams[k] parameters (0 for an aggregate node) written back to back into params.  A string without a composed
 * aggregate gives one node.  Every "Aggregate(...)" of a string is the runtime aggregatebsdf, as in the reference:
 * composed ones are BBM_HIP_AGGREGATE_BSDF nodes, fused ones carry BBM_HIP_RUNTIME_AGGREGATE in their id (in
 * bbm_hip_parse_model too).  Returns the node count or an error code. */
int bbm_hip_parse_model_tree(const char* str, int* model_ids, int* nchildren, float* params, int* nparams,
                             int max_nodes, int params_capacity);

/* ---------------------------------------------------------------- device scratch */

/* Return every idle block of the library's stream-ordered scratch pool (per-launch temporaries: sampler CDFs,
 * composed aggregates' per-lane terms) to the device, after the work that last used it has completed.  The pool
 * also frees idle blocks by itself beyond BBM_HIP_SCRATCH_RETAIN_MB (default 1024) of retained memory and when
 * an allocation fails.  Returns the bytes freed. */
size_t bbm_hip_scratch_trim(void);
/* Blocks handed out while the launch stream was capturing a HIP graph belong to that graph: the pool never reuses
 * or frees them (a replay writes to them), and neither bbm_hip_scratch_trim nor the pool's own trimming touches
 * them.  Once every such graph is destroyed, this frees them too (after a device synchronisation) and then trims
 * like bbm_hip_scratch_trim.  Calling it while a graph that used library scratch may still replay is an error
 * the library cannot detect.  Returns the bytes freed. */
size_t bbm_hip_scratch_trim_captured(void);
/* Bytes the pool currently holds (idle + in use). */
size_t bbm_hip_scratch_bytes(void);

/* ---------------------------------------------------------------- fitting (BASELINE config 5) */

/* Linearizer: a bijection between an index range [0, size) and (in, out) direction pairs
 * (concepts/inout_linearizer.h).  kind BBM_LIN_SPHERICAL = spherical_linearizer
 * (include/linearizer/spherical_linearizer.h:25-111): (phi, theta) grids of samples_in / samples_out
 * points over [start, end] (theta end points included); kind BBM_LIN_MERL = merl_linearizer
 * (include/linearizer/merl_linearizer.h:21-131): samples_in = samplesH (1, 90), samples_out =
 * samplesD (180, 90) in (phi, theta) order -- theta_h quadratic, theta_d / phi_d linear, start/end
 * unused. */
#define BBM_LIN_SPHERICAL 0
#define BBM_LIN_MERL 1
typedef struct bbm_hip_linearizer
{
  int32_t kind;
  uint64_t samples_in[2];
  uint64_t samples_out[2];
  float start_in[2], end_in[2], start_out[2], end_out[2];   /* (phi, theta), radians */
} bbm_hip_linearizer;

/* Number of direction pairs of the linearizer (linearizer::size()). */
int bbm_hip_linearizer_size(const bbm_hip_linearizer* lin, uint64_t* size);

/* Direction pairs begin .. begin + n - 1 of the linearizer into device SoA arrays. */
int bbm_hip_linearize(const bbm_hip_linearizer* lin, uint64_t begin, size_t n,
                      float* in_x, float* in_y, float* in_z, float* out_x, float* out_y, float* out_z,
                      void* stream);

/* Sample losses (include/loss/cosine_weighted_l2.h, include/loss/cosine_weighted_log.h) */
#define BBM_LOSS_NGAN_L2 0
#define BBM_LOSS_LOW_L2 1
#define BBM_LOSS_BIERON_L2 2
#define BBM_LOSS_STANDARD_LOG 3
#define BBM_LOSS_LOW_LOG 4
#define BBM_LOSS_BIERON_LOG 5

/* Workspace (bytes, device memory) bbm_hip_loss needs for nprobes probes. */
size_t bbm_hip_loss_workspace_size(int nprobes);

/* Multi-probe sampled loss -- sampledlossfunction::operator()() (include/bbm/sampledlossfunction.h:62-87)
 * for nprobes parameter vectors at once (a compass step's 2P probes, include/optimizer/compass.h:82-140),
 * over the samples begin .. begin + n - 1 of the linearizer (one GPU's shard):
 *   sums[p] = sum_i loss(in_i, out_i, model(probes[p]).eval(in_i, out_i, component, unit), ref_i)
 * accumulated in double; the caller divides by the linearizer size after summing the shards
 * (RCCL all-reduce).  probes: device, nprobes x nparams floats; ref_r/g/b: device, the reference
 * value of sample begin + i at [i]; sums: device, nprobes doubles; workspace: device,
 * bbm_hip_loss_workspace_size(nprobes) bytes.  Deterministic (fixed reduction order). */
int bbm_hip_loss(int model_id, const float* probes, int nparams, int nprobes,
                 const bbm_hip_linearizer* lin, uint64_t begin, size_t n,
                 const float* ref_r, const float* ref_g, const float* ref_b,
                 int loss_kind, uint32_t component, uint32_t unit,
                 double* sums, void* workspace, size_t workspace_bytes, void* stream);

/* bbm_hip_loss over n caller-provided direction pairs (a linearizer materialised once, e.g. with
 * bbm_hip_linearize, or any table of measured directions): the pair of sample i is (in[i], out[i]) and its
 * reference value ref[i].  Same probes / sums / workspace conventions as bbm_hip_loss; the fitting loop
 * reads 36 B per sample per pass instead of recomputing the linearizer's trigonometry. */
int bbm_hip_loss_pairs(int model_id, const float* probes, int nparams, int nprobes, size_t n,
                       const float* in_x, const float* in_y, const float* in_z,
                       const float* out_x, const float* out_y, const float* out_z,
                       const float* ref_r, const float* ref_g, const float* ref_b,
                       int loss_kind, uint32_t component, uint32_t unit,
                       double* sums, void* workspace, size_t workspace_bytes, void* stream);

/* The fitting loss of ANY model -- a single registry model, a fused or composed aggregate of either kind, nested to
 * any depth -- in floatRGB or doubleRGB (sampledlossfunction<BSDF, ...> takes any bsdfmodel and any configuration,
 * include/bbm/sampledlossfunction.h:34, :62-87), over n caller-provided pairs as bbm_hip_loss_pairs.  The model is a
 * child tree (bbm_hip_aggregate_*: a single model is one leaf node, ntree = 1) whose structure is used and whose
 * leaves' parameters are replaced, probe by probe, by the probe vectors: probes are HOST memory, nprobes x nparams
 * values, each the leaves' parameter vectors back to back in preorder.  Every probe is evaluated through the
 * model's kernels (composed aggregates: one pass per child) into device scratch and reduced per workgroup; sums as
 * bbm_hip_loss (device, nprobes doubles; f64: the per-sample losses in double throughout).  Workspace:
 * bbm_hip_loss_tree_workspace_size(nprobes, n) bytes of device memory. */
size_t bbm_hip_loss_tree_workspace_size(int nprobes, size_t n);
int bbm_hip_loss_tree(const bbm_hip_child* tree, int ntree, const float* probes, int nparams, int nprobes, size_t n,
                      const float* in_x, const float* in_y, const float* in_z,
                      const float* out_x, const float* out_y, const float* out_z,
                      const float* ref_r, const float* ref_g, const float* ref_b,
                      int loss_kind, uint32_t component, uint32_t unit,
                      double* sums, void* workspace, size_t workspace_bytes, void* stream);
int bbm_hip_loss_tree_f64(const bbm_hip_child_f64* tree, int ntree, const double* probes, int nparams, int nprobes,
                          size_t n, const double* in_x, const double* in_y, const double* in_z,
                          const double* out_x, const double* out_y, const double* out_z,
                          const double* ref_r, const double* ref_g, const double* ref_b,
                          int loss_kind, uint32_t component, uint32_t unit,
                          double* sums, void* workspace, size_t workspace_bytes, void* stream);

/* bbm::batch (include/bbm/batch.h:27-92): the loss over a random subset of a sampled loss's samples, redrawn by each
 * update().  Its indices come from bbm::rng<Size_t> (backbone/native/include/backbone/random.h:40-66: std::mt19937_64
 * and std::uniform_int_distribution<Size_t> over [lower, upper], both ends included), restated here on the host so a
 * batch holds the reference's indices for the same seed: batch(batchsize, loss, seed) is
 *   bbm_hip_rng_init(&rng, seed, 0, loss.samples()) then, per update(), bbm_hip_rng_draw(&rng, index, batchsize)
 * (batch.h:40-54; the upper end is the sample count itself, an index the sampled loss masks to 0, :65-66).
 * Caller-owned state, host only. */
typedef struct bbm_hip_rng
{
  uint64_t mt[312];
  uint64_t pos;
  uint64_t lower, upper;
  uint64_t magic;                          /* BBM_HIP_RNG_MAGIC once bbm_hip_rng_init has run; draw rejects others */
} bbm_hip_rng;
#define BBM_HIP_RNG_MAGIC 0x62626d726e673132ull
int bbm_hip_rng_init(bbm_hip_rng* rng, uint64_t seed, uint64_t lower, uint64_t upper);
int bbm_hip_rng_draw(bbm_hip_rng* rng, uint64_t* out, size_t n);     /* out: host memory */
/* The default seed of bbm::rng (std::mt19937_64::default_seed) */
#define BBM_HIP_RNG_DEFAULT_SEED 5489u

/* A batch's samples, gathered densely in draw order: dst[k][j] = src[k][index[i]] over the i with index[i] < nsamples
 * (a larger index is the reference's masked lane, which adds 0), for narrays (<= 16) device arrays of nsamples values
 * -- e.g. the materialised pairs (in xyz, out xyz) and reference table (r, g, b) of a fit.  index: HOST memory (the
 * drawn indices); src / dst: host arrays of device pointers, dst arrays with room for count values.  Any loss entry
 * point then scores the batch (bbm_hip_loss_pairs / _tree / _tree_f64 on the first n = returned count pairs).
 * Returns the number of samples gathered (>= 0) or an error code; returns after the gather has completed. */
int bbm_hip_gather_samples(const uint64_t* index, size_t count, uint64_t nsamples, const float* const* src,
                           float* const* dst, int narrays, void* stream);
int bbm_hip_gather_samples_f64(const uint64_t* index, size_t count, uint64_t nsamples, const double* const* src,
                               double* const* dst, int narrays, void* stream);

/* RCCL for the loss reduction of a fit sharded over GPUs (one process per GPU): each rank scores every probe of a
 * compass step on its shard (bbm_hip_loss* -> sums), then the nprobes double sums are all-reduced in place (RCCL over
 * xGMI, ncclSum on ncclFloat64) and every rank takes the same compass decision (include/optimizer/compass.h:122-126).
 * Rank 0 makes the unique id (bbm_hip_comm_unique_id) and hands its bytes to the other ranks by any means (MPI, a
 * file, a torch.distributed broadcast); every rank then calls bbm_hip_comm_init on its own current HIP device.
 * librccl is loaded on first use (BBM_HIP_ERR_UNSUPPORTED without it). */
#define BBM_HIP_COMM_ID_BYTES 128
typedef struct bbm_hip_comm bbm_hip_comm;
int bbm_hip_comm_unique_id(uint8_t* id, size_t bytes);
int bbm_hip_comm_init(const uint8_t* id, size_t bytes, int rank, int world, bbm_hip_comm** comm);
int bbm_hip_comm_destroy(bbm_hip_comm* comm);
int bbm_hip_comm_rank(const bbm_hip_comm* comm);
int bbm_hip_comm_size(const bbm_hip_comm* comm);
/* sums[0 .. n-1] (device doubles) <- their sum over all ranks, on `stream` */
int bbm_hip_allreduce_sums(bbm_hip_comm* comm, double* sums, size_t n, void* stream);

/* The EPD model's shadowing table G1[p][t] (100 x 1000 floats, row-major; the reference's
 * include/precomputed/holzschuchpacanowski/G1.h), built on the current device on first use by
 * restating its generator (precompute/HolzschuchPacanowski/G1.cpp).  Copies min(capacity, 100000)
 * entries to host memory `out` (may be NULL) and returns the table size, or a negative error code. */
int bbm_hip_epd_g1_table(float* out, int capacity);

/* Merl (include/staticmodel/merl.h): build the model's device table from a MERL-MIT .binary file.
 * Replaces merl_data::import (merl.h:173-206).  `raw` = device copy of the 3 x theta_h x theta_d x phi_d
 * doubles that follow the file's three uint32 dimensions (channel planes R, G, B); `table` = device
 * buffer of theta_h*theta_d*phi_d float4 (16 B) entries, filled with (max(0, R/1500), max(0, 1.15 G/1500),
 * max(0, 1.66 B/1500), 0) rounded to float.  Dimensions other than 90 x 90 x 180 are rejected as in the
 * reference.  The Merl model's two parameters are the table's device address (low, high 32 bits). */
#define BBM_HIP_MERL_ENTRIES (90u * 90u * 180u)
int bbm_hip_merl_table(const double* raw, uint32_t theta_h, uint32_t theta_d, uint32_t phi_d, float* table,
                       void* stream);

/* ---------------------------------------------------------------- synthetic directions */

/* Fill n directions from a counter-based generator: element i depends only on (seed, offset + i),
 * so shards on different GPUs regenerate their slice of one global batch without any scatter.
 * mode 0: uniform in z on the upper hemisphere (z = u, phi = 2 pi u'), the worst case with every
 * lane active; mode 1: uniform on the sphere (bin/checkBsdf.cpp:28-35 sampleSphere).
 * stream_id selects an independent stream of the generator (e.g. 0 = in, 1 = out). */
int bbm_hip_fill_directions(uint64_t seed, uint32_t stream_id, uint64_t offset, size_t n, int mode,
                            float* x, float* y, float* z, void* stream);

/* ---------------------------------------------------------------- checkBsdf statistics */

/* bin/checkBsdf.cpp's tests (:51-418) as batched reductions over n random samples per slot.
 * Random numbers: counter-based (bbm_hip_check_draws), one stream per (test, slot, draw), so a
 * shard [begin, begin + n) of the samples draws exactly what one GPU would have drawn for them.
 * Accumulators are double; acc (device) receives nslots x BBM_CHECK_ACC doubles, laid out per test:
 *   REFLECTANCE (:51-97)   slot = theta_out (slot direction = out): [0..2] sum eval(dir, out) z(dir) / pdf,
 *                          [3] accepted samples (pdf > eps); importance != 0 samples the BSDF, else sampleSphere
 *   RECIPROCITY (:102-140) [0..2] sum |f(in,out) - f(out,in)| Radiance, [3..5] Importance,
 *                          [8] max hsum (Radiance) at sample [9], [10] max hsum (Importance) at sample [11]
 *   ADJOINT (:145-185)     [0..2] sum |f_Radiance(in,out) - f_Importance(out,in)|, [8] max hsum at sample [9]
 *   PDF (:190-245)         [0]/[1] negative pdf (Radiance/Importance), [2]/[3] sampled below the horizon,
 *                          [4]/[5] sum |sample.pdf - pdf(sample.direction, out)|; out on the hemisphere
 *                          (sphere != 0: sphere)
 *   PDFINT (:250-290)      slot = trial (slot direction = trial direction): [0]/[1] sum pdf(dir, t) / (1 / 4 pi)
 *   SAMPLE_PDF (:330-357)  slot = trial * bins + bin (slot directions = trial directions, one per trial):
 *                          [0] sum pdf(dir, t) * solid angle weight over the bin's n pdf samples
 *   SAMPLE_COUNT (:360-380) slot = trial: counts[slot][bin] = samples landing in the (theta, phi) bin
 *                          (pdf > eps unless include_zero_pdf); acc unused, counts zeroed by the call.
 * The caller divides by the sample counts (after summing shards across GPUs). */
#define BBM_CHECK_REFLECTANCE 0
#define BBM_CHECK_RECIPROCITY 1
#define BBM_CHECK_ADJOINT 2
#define BBM_CHECK_PDF 3
#define BBM_CHECK_PDFINT 4
#define BBM_CHECK_SAMPLE_PDF 5
#define BBM_CHECK_SAMPLE_COUNT 6
#define BBM_CHECK_ACC 12

typedef struct bbm_hip_check_desc
{
  int32_t test;
  int32_t nslots;
  uint64_t seed;
  uint64_t begin, n;                 /* samples [begin, begin + n) of every slot */
  const float* slot_x;               /* device, per-slot direction (see above); NULL where unused */
  const float* slot_y;
  const float* slot_z;
  int32_t sphere;                    /* PDF: out uniform on the sphere instead of the hemisphere */
  int32_t importance;                /* REFLECTANCE: importance sampling */
  int32_t include_zero_pdf;          /* SAMPLE_COUNT: includeZeroPdfSamples */
  uint32_t theta_bins, phi_bins;     /* SAMPLE_PDF / SAMPLE_COUNT */
} bbm_hip_check_desc;

/* Workspace (bytes, device memory) bbm_hip_check needs for this descriptor. */
size_t bbm_hip_check_workspace_size(const bbm_hip_check_desc* desc);

/* Run one checkBsdf statistic of model_id (params uniform) -> acc / counts (device). */
int bbm_hip_check(int model_id, const float* params, int nparams, const bbm_hip_check_desc* desc,
                  double* acc, uint64_t* counts, void* workspace, size_t workspace_bytes, void* stream);

/* checkBsdf for ANY model (a child tree as in bbm_hip_loss_tree, leaves with their own parameters; checkBsdf builds
 * any model string through bsdf_import, bin/checkBsdf.cpp:435-479) and for doubleRGB.  The same tests, draws, slot
 * semantics, accumulator layout and fixed-order final reduction as bbm_hip_check; the per-sample quantities are
 * materialised in chunks through the model's own sample / eval / pdf entry points (composed aggregates: one pass per
 * child) and reduced per chunk.  f64: every per-sample quantity in double (sampleSphere, the chi-square points and
 * bins in double), the slot directions given as doubles (the descriptor's float slot pointers are ignored).
 * Workspace: bbm_hip_check_tree_workspace_size(desc) bytes of device memory (0 for SAMPLE_COUNT). */
size_t bbm_hip_check_tree_workspace_size(const bbm_hip_check_desc* desc);
int bbm_hip_check_tree(const bbm_hip_child* tree, int ntree, const bbm_hip_check_desc* desc, double* acc,
                       uint64_t* counts, void* workspace, size_t workspace_bytes, void* stream);
int bbm_hip_check_tree_f64(const bbm_hip_child_f64* tree, int ntree, const bbm_hip_check_desc* desc,
                           const double* slot_x, const double* slot_y, const double* slot_z, double* acc,
                           uint64_t* counts, void* workspace, size_t workspace_bytes, void* stream);

/* The uniforms draw `draw` (0..2) of slot `slot` of `test` uses for samples offset .. offset + n - 1
 * (rndVec2d(), checkBsdf.cpp:21-26): xi0[i], xi1[i] in [0, 1), 24-bit. */
int bbm_hip_check_draws(int test, uint64_t seed, int slot, int draw, uint64_t offset, size_t n,
                        float* xi0, float* xi1, void* stream);

/* Trial directions of PDFINT / SAMPLE_PDF / SAMPLE_COUNT: trial t = sampleHemisphere (sphere = 0) or
 * sampleSphere (sphere != 0) of its own draw (checkBsdf.cpp:270, :322). */
int bbm_hip_check_trials(int test, uint64_t seed, int ntrials, int sphere, float* x, float* y, float* z, void* stream);

/* sampleSphere / sampleHemisphere (checkBsdf.cpp:28-45) of n uniform pairs (device). */
int bbm_hip_sphere_dirs(const float* xi0, const float* xi1, size_t n, int hemisphere, float* x, float* y, float* z,
                        void* stream);

/* ---------------------------------------------------------------- device math verification */

/* The device restatements of the host libm float functions the reference's native backbone calls (glibc 2.35's
 * expf, logf, powf, erff, erfcf, sinf, cosf, atan2f: bbm_amd/csrc/math.hpp), evaluated elementwise on n device floats:
 * out[i] = f(a[i]) (f(a[i], b[i]) for powf, ONE_PLUS_SQRT, atan2f, THETA; b may be NULL otherwise).  For pinning them against the host libm on
 * the machine that runs the reference (tests/test_gpu_libm.py); not on any BSDF path. */
#define BBM_HIP_LIBM_EXPF 0
#define BBM_HIP_LIBM_LOGF 1
#define BBM_HIP_LIBM_POWF 2
#define BBM_HIP_LIBM_ERFF 3
#define BBM_HIP_LIBM_ERFCF 4
#define BBM_HIP_LIBM_ONE_PLUS_SQRT 5   /* float(1.0 + sqrt(1.0 + (double)a * b)), the GGX G1 denominator */
#define BBM_HIP_LIBM_SINF 6
#define BBM_HIP_LIBM_COSF 7
#define BBM_HIP_LIBM_ATAN2F 8       /* atan2f(a, b) */
#define BBM_HIP_LIBM_THETA 9        /* spherical::theta of the direction (a, 0, b): float(2 asin(|v - pole| / 2)) */
int bbm_hip_libm_eval(int func, const float* a, const float* b, float* out, size_t n, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* BBM_HIP_H */
