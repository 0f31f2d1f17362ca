/*
 * mha_hd64.h — C ABI of the MI355X-native MHAHeadDim64 attention operator.
 *
 * This is the drop-in boundary for the hot path of
 * qdLMF/LightGlue-with-FlashAttentionV2-TensorRT: the fused FlashAttention-v2
 * head_dim=64 self/cross attention that LightGlue calls 36 times per image pair.
 *
 * The reference exposes the operator as a TensorRT IPluginV2DynamicExt
 * ("MHAHeadDim64", version "1",
 *  lightglue_attention_plugin/lightglue_attention_plugin.h:28-121, impl
 *  lightglue_attention_plugin/lightglue_attention_plugin.cpp:28-359) plus an
 * IPluginCreator (.h:125-159, .cpp:363-420). Every virtual method of that
 * plugin that the engine calls is exported below as a plain C function taking
 * an opaque plugin handle, plain structs, pointers and sizes (no TensorRT, no
 * torch types). A host that used to dlopen the TRT plugin binds these symbols
 * instead (see INTEGRATION.md for the ctypes / C++ bindings).
 *
 * The kernel launchers of the reference's L0 layer
 * (AttentionHeadDim64::launch_* in attention_headdim_64_fp16in_fp16out.cuh:17-57
 *  and attention_headdim_64_fp16in_fp32out.cuh:18-76) are exported too, as
 * mha_hd64_launch_*; they need no plugin object.
 *
 * Errors: the reference's PLUGIN_ASSERT logs, calls cudaDeviceReset() and
 * abort()s (common/checkMacrosPlugin.cpp:118-128). Through a C ABI we return a
 * nonzero MHA_HD64_STATUS_* code instead and record a message readable with
 * mha_hd64_last_error(). mha_hd64_set_abort_on_error(1) restores the
 * reference's abort-on-assert behaviour (without the device reset).
 *
 * Threading: the plugin object is stateless apart from its namespace string.
 * Concurrent enqueues on different streams are safe when their workspaces
 * differ (same rule as the reference, .cpp:172-175). The library keeps one
 * small arrival-ticket array per (device, stream) and a per-device arena for
 * launches recorded under stream capture (see mha_hd64_enqueue).
 */
#ifndef MHA_HD64_H
#define MHA_HD64_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Compile-time limits, identical to lightglue_attention_plugin.h:19-22. */
#define MHA_HD64_BATCH        1
#define MHA_HD64_NUM_HEADS    4
#define MHA_HD64_MAX_SEQ_LEN  2048
#define MHA_HD64_HEAD_DIM     64

/* Status codes (0 = success, the reference's enqueue() return value). */
#define MHA_HD64_STATUS_SUCCESS        0
#define MHA_HD64_STATUS_BAD_PARAM      1   /* a PLUGIN_ASSERT would have fired  */
#define MHA_HD64_STATUS_LAUNCH_FAILED  2   /* hipGetLastError() after a launch   */
#define MHA_HD64_STATUS_WORKSPACE      3   /* workspace too small for the call   */

/* Values mirror nvinfer1::DataType (kFLOAT = 0, kHALF = 1). */
typedef enum { MHA_HD64_DT_FLOAT = 0, MHA_HD64_DT_HALF = 1 } mha_hd64_dtype_t;
/* Values mirror nvinfer1::TensorFormat (kLINEAR = 0). */
typedef enum { MHA_HD64_FMT_LINEAR = 0 } mha_hd64_format_t;

/* Mirrors nvinfer1::Dims (MAX_DIMS = 8). */
typedef struct {
    int32_t nb_dims;
    int64_t d[8];
} mha_hd64_dims_t;

/* Mirrors nvinfer1::PluginTensorDesc. */
typedef struct {
    mha_hd64_dims_t dims;
    int32_t type;     /* mha_hd64_dtype_t  */
    int32_t format;   /* mha_hd64_format_t */
    float scale;
} mha_hd64_tensor_desc_t;

/* Mirrors nvinfer1::DynamicPluginTensorDesc. */
typedef struct {
    mha_hd64_tensor_desc_t desc;
    mha_hd64_dims_t min;
    mha_hd64_dims_t max;
} mha_hd64_dynamic_tensor_desc_t;

typedef struct mha_hd64_plugin mha_hd64_plugin_t;

/* ---- creator (IPluginCreator, lightglue_attention_plugin.cpp:363-420) ---- */
const char* mha_hd64_creator_plugin_name(void);        /* getPluginName    .cpp:371-373 -> "MHAHeadDim64" */
const char* mha_hd64_creator_plugin_version(void);     /* getPluginVersion .cpp:375-377 -> "1"            */
int32_t     mha_hd64_creator_nb_fields(void);          /* getFieldNames    .cpp:387-389 -> 0 fields        */
mha_hd64_plugin_t* mha_hd64_create_plugin(const char* name);                   /* createPlugin .cpp:391-404 */
mha_hd64_plugin_t* mha_hd64_deserialize_plugin(const char* name, const void* data,
                                               size_t length);                 /* deserializePlugin .cpp:406-420 */

/* ---- plugin (IPluginV2DynamicExt, lightglue_attention_plugin.cpp:28-359) ---- */
void        mha_hd64_destroy(mha_hd64_plugin_t* p);                          /* destroy     .cpp:41-43  */
mha_hd64_plugin_t* mha_hd64_clone(const mha_hd64_plugin_t* p);               /* clone       .cpp:65-75  */
int32_t     mha_hd64_initialize(mha_hd64_plugin_t* p);                       /* initialize  .cpp:36      */
void        mha_hd64_terminate(mha_hd64_plugin_t* p);                        /* terminate   .cpp:38-39  */
size_t      mha_hd64_get_serialization_size(const mha_hd64_plugin_t* p);     /* .cpp:45 -> 0             */
void        mha_hd64_serialize(const mha_hd64_plugin_t* p, void* buffer);    /* .cpp:47 (no state)      */
const char* mha_hd64_get_plugin_type(const mha_hd64_plugin_t* p);            /* .cpp:49                  */
const char* mha_hd64_get_plugin_version(const mha_hd64_plugin_t* p);         /* .cpp:51                  */
void        mha_hd64_set_plugin_namespace(mha_hd64_plugin_t* p, const char* ns); /* .cpp:53            */
const char* mha_hd64_get_plugin_namespace(const mha_hd64_plugin_t* p);       /* .cpp:55                  */
void        mha_hd64_attach_to_context(mha_hd64_plugin_t* p);                /* .cpp:57-61 (no-op)       */
void        mha_hd64_detach_from_context(mha_hd64_plugin_t* p);              /* .cpp:63 (no-op)          */
int32_t     mha_hd64_get_nb_outputs(const mha_hd64_plugin_t* p);             /* .cpp:77 -> 1             */

/* getOutputDimensions (.cpp:79-94): out = inputs[0]. Returns a status. */
int32_t mha_hd64_get_output_dimensions(mha_hd64_plugin_t* p, int32_t output_index,
                                       const mha_hd64_dims_t* inputs, int32_t nb_inputs,
                                       mha_hd64_dims_t* out);

/* supportsFormatCombination (.cpp:272-296): 1 = supported, 0 = not, <0 = bad call. */
int32_t mha_hd64_supports_format_combination(mha_hd64_plugin_t* p, int32_t pos,
                                             const mha_hd64_tensor_desc_t* in_out,
                                             int32_t nb_inputs, int32_t nb_outputs);

/* getOutputDataType (.cpp:298-310): *out_type = inputs_type[0]. Returns a status. */
int32_t mha_hd64_get_output_data_type(const mha_hd64_plugin_t* p, int32_t output_index,
                                      const int32_t* inputs_type, int32_t nb_inputs,
                                      int32_t* out_type);

/* configurePlugin (.cpp:312-359): validation only. Returns a status. */
int32_t mha_hd64_configure_plugin(mha_hd64_plugin_t* p,
                                  const mha_hd64_dynamic_tensor_desc_t* in, int32_t nb_inputs,
                                  const mha_hd64_dynamic_tensor_desc_t* out, int32_t nb_outputs);

/* getWorkspaceSize (.cpp:96-112): fixed 5,242,880 B, independent of N, as in the reference. */
size_t mha_hd64_get_workspace_size(const mha_hd64_plugin_t* p,
                                   const mha_hd64_tensor_desc_t* in, int32_t nb_inputs,
                                   const mha_hd64_tensor_desc_t* out, int32_t nb_outputs);

/* enqueue (.cpp:114-270). Same asserts as configurePlugin; dispatch on in[0].type:
 *   HALF  -> fp16 in, fp32 accumulation, fp16 out   (reference: pad -> fp16in_fp16out kernel -> unpad)
 *   FLOAT -> fp32 in rounded to fp16 (RN) on load, fp32 accumulation, fp32 out
 *            (reference: convert+pad -> fp16in_fp32out kernel -> unpad)
 * One kernel launch on `stream`. At the reference's shapes with N <= 2048 (HALF) a workgroup
 * holds all keys of its 16 query rows (the 16-row single-pass kernel: 256 workgroups for a
 * 1x4x1024x1024 call, no split, no workspace use; 32-row blocks under a concurrency hint >= 2;
 * FLOAT with N <= 1024 rounds fp32 to fp16 inside the same kernel, one launch). A call
 * whose keys are split across workgroups merges the
 * splits inside that launch through library-owned arrival tickets; the first enqueue on a
 * (device, stream) outside stream capture allocates them (and, once per device, a pre-zeroed
 * arena for captured launches, with one stream sync). Without tickets (first use of a stream
 * inside a capture, env MHA_HD64_FUSED_COMBINE=0) a second, combine kernel does the merge; the
 * results are bitwise identical. `workspace` must hold mha_hd64_get_workspace_size() bytes.
 * Returns a status. */
int32_t mha_hd64_enqueue(mha_hd64_plugin_t* p,
                         const mha_hd64_tensor_desc_t* in, const mha_hd64_tensor_desc_t* out,
                         const void* const* inputs, void* const* outputs,
                         void* workspace, hipStream_t stream);

/* ---- L0 kernel launchers (AttentionHeadDim64::launch_*) ----
 * Q [batch, heads, nq, 64], K/V [batch, heads, nkv, 64], O [batch, heads, nq, 64],
 * all contiguous row-major. No padding requirements (tails are masked in-kernel,
 * which replaces the reference's pad/unpad helpers a4/a5/a7). workspace may be
 * NULL when ws_bytes == 0 (the launcher then runs without a KV split). */
int32_t mha_hd64_launch_fp16in_fp16out(const void* q, const void* k, const void* v, void* o,
                                       int32_t batch, int32_t heads, int32_t nq, int32_t nkv,
                                       void* workspace, size_t ws_bytes, hipStream_t stream);
int32_t mha_hd64_launch_fp16in_fp32out(const void* q, const void* k, const void* v, void* o,
                                       int32_t batch, int32_t heads, int32_t nq, int32_t nkv,
                                       void* workspace, size_t ws_bytes, hipStream_t stream);
int32_t mha_hd64_launch_fp32in_fp32out(const void* q, const void* k, const void* v, void* o,
                                       int32_t batch, int32_t heads, int32_t nq, int32_t nkv,
                                       void* workspace, size_t ws_bytes, hipStream_t stream);

/* Workspace bytes the launchers can use to split the KV range of a call of
 * this shape across workgroups (0 = the call never splits). fp16 inputs. */
size_t mha_hd64_launch_workspace_bytes(int32_t batch, int32_t heads, int32_t nq, int32_t nkv);
/* The same for inputs of in_type (mha_hd64_dtype_t). For FLOAT inputs that the planner runs as a
 * convert launch + an fp16 single-pass kernel this includes the fp16 copies of Q/K/V; with less
 * workspace mha_hd64_launch_fp32in_fp32out takes the ring kernel rounding on load instead (same
 * results within the tolerance, up to ~1.8x slower at 1x4x1024x2048). 0 for an invalid in_type. */
size_t mha_hd64_launch_workspace_bytes_typed(int32_t batch, int32_t heads, int32_t nq, int32_t nkv,
                                             int32_t in_type);

/* ---- grouped launcher ----
 * Several independent calls of (possibly) different shapes in one launch. A LightGlue layer
 * makes four attention calls whose inputs are all ready together: SelfBlock on image 0 and on
 * image 1 (lightglue_pytorch_with_plugin/lightglue.py:137-152, Nq = Nkv = N0 and N1) and the
 * two CrossBlock directions (lightglue.py:188-205, N0 x N1 and N1 x N0); the reference runs
 * each as its own plugin enqueue (four kernel chains per layer, TransformerLayer :216-226).
 * Up to 4 calls share one launch (split keys are merged inside it, as for enqueue); longer
 * lists are chunked. All calls use one dtype pair:
 *   in_type HALF  -> fp16 inputs; FLOAT -> fp32 inputs rounded to fp16 on load
 *   out_type HALF -> fp16 output; FLOAT -> fp32 output
 * Same per-call layout rules as the L0 launchers. Returns a status. */
typedef struct mha_hd64_call {
    const void* q;
    const void* k;
    const void* v;
    void* o;
    int32_t batch;
    int32_t heads;
    int32_t nq;
    int32_t nkv;
} mha_hd64_call_t;

int32_t mha_hd64_launch_grouped(const mha_hd64_call_t* calls, int32_t n_calls, int32_t in_type,
                                int32_t out_type, void* workspace, size_t ws_bytes, hipStream_t stream);
/* Workspace bytes the grouped launcher can use for fp16 inputs (0 = no call of the group splits). */
size_t mha_hd64_grouped_workspace_bytes(const mha_hd64_call_t* calls, int32_t n_calls);
/* The same for inputs of in_type (mha_hd64_dtype_t): for FLOAT groups that a single-pass kernel
 * runs after a convert launch this includes the fp16 copies of Q/K/V; with less workspace such
 * groups take the slower ring kernel (convert on load). The largest chunk of 4 calls counts
 * (chunks reuse the workspace in stream order). 0 for an invalid in_type. */
size_t mha_hd64_grouped_workspace_bytes_typed(const mha_hd64_call_t* calls, int32_t n_calls, int32_t in_type);

/* ---- concurrency hint (no reference counterpart: TensorRT gives a plugin no view of its
 * other streams) ----
 * How many independent enqueue streams the host keeps busy on this process's GPUs at once
 * (independent image pairs, one stream each). 1 (default): every call
 * may take the whole chip, so a 1x4x1024x1024 call runs on 256 workgroups of 16 query rows, one
 * per CU. 2: calls take half the chip (128 workgroups of 32 rows) so two streams' calls run side
 * by side. >= 3: the same 32-row blocks in the two-per-CU form (65 KiB of LDS each), so up to
 * four calls share the chip. Results are identical in every mode up to fp32 summation order
 * (each mode is deterministic). Returns the previous hint; values < 1 read as 1. Process-wide. */
int32_t mha_hd64_set_concurrency_hint(int32_t streams);

/* ---- kernel-form switches (no reference counterpart; process-wide, thread-safe, take effect at
 * the next launch; every setting gives results within the same tolerance of the oracle) ---- */
/* Throughput kernel for launches that carry more than one round of 128-row query blocks (batched
 * image-pair streams, grouped layers of several pairs): 1 (default) = the persistent streaming
 * kernel (fp16 inputs), 0 = the LDS-ring kernel. The environment variable
 * MHA_HD64_STREAM=0/1 sets the initial value. Returns the previous mode. */
int32_t mha_hd64_set_stream_mode(int32_t mode);
/* FLOAT (fp32) inputs: 1 (default) = rounded to fp16 inside the attention kernel where that
 * measured faster (one launch), 0 = always a convert launch into the workspace + the fp16 kernel,
 * 2 = also the two-pass in-kernel forms (1024 < nkv <= 2048; diagnostic, measured slower).
 * Outputs are bitwise identical in every mode. Env MHA_HD64_F32_INKERNEL sets the initial value. */
void mha_hd64_set_f32_inkernel(int32_t mode);
/* Calls whose keys are split across workgroups: 1 (default) = merged inside the launch through
 * library-owned arrival tickets, 0 = a second (combine) kernel. Bitwise-identical results. */
void mha_hd64_set_fused_combine(int32_t enable);

/* ---- diagnostics ---- */
const char* mha_hd64_last_error(void);           /* thread-local message of the last failure   */
void        mha_hd64_set_abort_on_error(int32_t enable); /* 1 = abort() like PLUGIN_ASSERT     */
const char* mha_hd64_build_info(void);           /* target arch, compiler, kernel variants      */

/* ---- test and benchmark hooks (exported for tests/, tools/ and bench.py; not needed by a
 * plugin host, no stability promise) ---- */
/* Launch with a forced kernel form: q_waves/kv_waves/splits as the planner's fields (0 = the
 * planner's choice); q_waves 21 / 22 / 23 force the 32-row / 16-row single-pass kernel / the
 * streaming kernel (with q_waves 23, kv_waves 4 or 8 picks its 4- or 8-wave form, 0 the planner's).
 * phase_mask: 1 main kernel only, 2 combine only, 3 both. Returns a status
 * (BAD_PARAM when the form is not compiled for the shape). */
int32_t mha_hd64_launch_forced(const void* q, const void* k, const void* v, void* o, int32_t batch, int32_t heads,
                               int32_t nq, int32_t nkv, int32_t in_f32, int32_t out_f32, int32_t q_waves,
                               int32_t kv_waves, int32_t splits, void* workspace, size_t ws_bytes,
                               hipStream_t stream, int32_t phase_mask);
/* The planner's choice for a fp16 call: out4 = {q_waves (or 21/22/23), kv_waves, splits,
 * tiles_per_split} (streaming plan: {23, 4 or 8 waves, 1, ...}); returns the workspace bytes that
 * plan uses. */
size_t mha_hd64_plan(int32_t batch, int32_t heads, int32_t nq, int32_t nkv, size_t ws_bytes, int32_t* out4);
/* Per-workgroup timestamp buffer of -DMHA_STAMPS diagnostic builds (ignored by release builds). */
void mha_hd64_set_stamp_buffer(void* p);
/* How the calling thread's last launch merged its KV splits: 0 no split, 1 in-launch, 2 kernel. */
int32_t mha_hd64_last_combine_form(void);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* MHA_HD64_H */
