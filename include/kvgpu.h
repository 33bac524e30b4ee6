/*
 * kvgpu.h — C ABI of the MI355X-native batch validate.pattern engine.
 *
 * Drop-in boundary for Kyverno's validate hot path (isabella232/kyverno v1.5.x):
 *   engine.Validate(policyContext *PolicyContext) *response.EngineResponse
 *       pkg/engine/validation.go:26
 * called per (policy, resource) by
 *   CLI apply        pkg/kyverno/common/common.go:541 (loop at pkg/kyverno/apply/apply_command.go:270-310)
 *   background scan  pkg/policy/apply.go:72 (via pkg/policy/existing.go:55-58)
 *   test runner      pkg/testrunner/scenario.go:169
 * The batch form evaluates every (resource, rule) pair of a policy set at once.
 * Plain C types only; all handles are opaque and library-owned until kv_free_*.
 * Return value: 0 on success, negative KV_E_* on failure (with *err set when
 * err != NULL; free with kv_free_error). Per-pair evaluation never fails: it
 * yields status KV_STATUS_ERROR exactly like the reference.
 */
#ifndef KVGPU_H
#define KVGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* response.RuleStatus (pkg/engine/response/status.go:14-28) + batch extras */
enum {
  KV_STATUS_PASS = 0,
  KV_STATUS_FAIL = 1,
  KV_STATUS_WARN = 2,
  KV_STATUS_ERROR = 3,
  KV_STATUS_SKIP = 4,
  KV_STATUS_NOMATCH = 5, /* no RuleResponse: rule not matched / not a pattern rule (CLI counts skip) */
  KV_STATUS_CPU = 6      /* route the pair to the reference CPU engine (processValidationRule) */
};

/* rule routes decided at compile time */
enum { KV_ROUTE_GPU = 0, KV_ROUTE_CPU = 1, KV_ROUTE_NORESPONSE = 2, KV_ROUTE_CONSTANT = 3 };

/* kv_compile flags */
enum {
  /* also lower every rule to a specialized gfx950 kernel (hiprtc, at compile
   * time); kv_validate/kv_session then run those instead of the bytecode VM */
  KV_COMPILE_SPECIALIZE = 1
};

/* kv_validate modes (bit set). KV_MODE_SCOPES adds per-scope counts
 * (scope = namespace; "" = cluster scope), the PolicyReport / ClusterPolicyReport
 * summaries of pkg/kyverno/apply/report.go:76-179 and the background controller's
 * pkg/policyreport/builder.go:245-308; the specialized kernels count them inside the
 * pass (no status matrix unless KV_MODE_STATUS / KV_MODE_ERRORS is asked for too). */
enum { KV_MODE_STATUS = 1, KV_MODE_ERRORS = 2, KV_MODE_COUNTS = 4, KV_MODE_SCOPES = 8 };

enum { KV_E_INVALID = -1, KV_E_PARSE = -2, KV_E_DEVICE = -3, KV_E_RANGE = -4, KV_E_NOMEM = -5 };

typedef struct kv_policyset kv_policyset;
typedef struct kv_batch kv_batch;
typedef struct kv_result kv_result;
typedef struct kv_error {
  int code;
  char* message;
} kv_error;

typedef struct kv_rule_info {
  uint32_t policy;          /* index of the policy in the compiled list */
  const char* policy_name;  /* metadata.name */
  const char* name;         /* rule name */
  uint32_t route;           /* KV_ROUTE_* */
  const char* route_reason; /* why CPU / no-response ("" for GPU) */
  const char* message;      /* validate.message */
  uint32_t any_pattern;     /* 1 for anyPattern rules */
  uint32_t const_status;    /* KV_ROUTE_CONSTANT */
  const char* const_message;
} kv_rule_info;

/* Compile a JSON list of ClusterPolicy/Policy objects (already through
 * policymutation autogen, as the reference CLI does before engine.Validate).
 * Replaces the per-call interpretation in pkg/engine/validate, pkg/engine/anchor,
 * pkg/engine/operator and the $() reference substitution of
 * pkg/engine/variables/vars.go:253-309. */
int kv_compile(const char* policies_json, size_t len, uint32_t flags, kv_policyset** out, kv_error** err);
int kv_policyset_info(const kv_policyset* ps, uint32_t* n_policies, uint32_t* n_rules);
/* specialized kernels of a KV_COMPILE_SPECIALIZE policy set (zeros otherwise) */
int kv_policyset_jit_info(const kv_policyset* ps, uint32_t* n_kernels, double* gen_ms, double* compile_ms,
                          uint64_t* code_bytes);
int kv_rule_info_get(const kv_policyset* ps, uint32_t rule, kv_rule_info* out);

/* Ingest resources (JSON array or NDJSON of unstructured objects; numbers typed
 * like unstructured.UnmarshalJSON). ns_labels_json: {"<namespace>": {"k":"v"}}
 * (PolicyContext.NamespaceLabels per namespace) or NULL. */
int kv_ingest(const kv_policyset* ps, const char* resources_json, size_t len, const char* ns_labels_json,
              kv_batch** out, kv_error** err);
int kv_batch_info(const kv_batch* b, uint64_t* n_res, uint64_t* store_bytes);
/* bytes the batch's store crosses PCIe in (kv_validate's upload: the populated cells in their
 * 8-byte transfer form, row masks, values, resource headers, strings, match inputs); no
 * reference counterpart (the reference evaluates in the process that decoded the resource) */
int kv_batch_transfer_bytes(const kv_batch* b, uint64_t* bytes);
/* namespace table of a batch (first-seen order; index = scope of kv_result_scope_counts);
 * the name lives as long as the batch. Reference: resource.GetNamespace() keys the report
 * scope in buildPolicyResults (pkg/kyverno/apply/report.go:80-87). */
int kv_batch_namespaces(const kv_batch* b, uint32_t* n);
const char* kv_batch_namespace(const kv_batch* b, uint32_t i);

/* Evaluate every (resource, rule) pair on HIP device `device`.
 * ctx_json: {"admission": {"roles":[], "clusterRoles":[], "groups":[], "username":""},
 *            "excludeGroupRole": []}  (PolicyContext.AdmissionInfo / ExcludeGroupRole) or NULL. */
int kv_validate(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, int device, uint32_t mode,
                kv_result** out, kv_error** err);

/* Evaluate on several devices (SURVEY.md §8b "Threading"): the batch's resources are
 * split into contiguous ranges [k*N/G, (k+1)*N/G) (cut at 64-resource boundaries)
 * over the G devices of device_mask (bit d = HIP device d), one host thread + HIP
 * stream per device, the policy set replicated; per-rule counts (and per-scope
 * counts with KV_MODE_SCOPES) are summed over the devices by one RCCL all-reduce
 * (ncclUint64, ncclSum; communicators created per session). Statuses and error
 * records come back in resource order in one result. Callers: the background
 * scan (pkg/policy/apply.go:72) and kyverno apply (pkg/kyverno/apply/apply_command.go:270-310). */
int kv_validate_devices(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, uint32_t device_mask,
                        uint32_t mode, kv_result** out, kv_error** err);

/* status[rule * n_res + res] (rule-major). The statuses of a specialized pass cross PCIe in a
 * transfer form (the 256-resource segments the pass wrote, 4 bits a status; the others NOMATCH);
 * the first call with a non-NULL `status` builds the dense matrix on the host threads (C3 1.25 M x
 * 1 973: ~60 ms) and later calls return it. status = NULL: dimensions only, nothing built. */
int kv_result_status(const kv_result* r, const uint8_t** status, uint64_t* n_rules, uint64_t* n_res);
/* counts[rule * 8 + status] */
int kv_result_counts(const kv_result* r, const int64_t** counts);
/* Page-lock `bytes` of host memory for the library's store and result arrays up front (once per
 * process; a later call only reports whether the reserve is at least that large), so the ingest of
 * a process's first batch and its first results find page-locked memory instead of pinning it
 * then. 0 on success, KV_E_DEVICE without a device or when the host refuses the memory. */
int kv_host_reserve(uint64_t bytes);
/* Device buffers released by batches, results and sessions are kept per device and handed to the
 * next allocation of a similar size (a released buffer is reused only after the work queued before
 * its release has finished). kv_device_pool_limit sets how many bytes are kept per device (default
 * 32 GiB; 0 keeps none); kv_device_trim frees what device `device` keeps now, e.g. before another
 * allocator in the process (torch) needs the memory. No reference counterpart (Go frees nothing
 * on a device). 0 on success, KV_E_DEVICE for a bad device. */
int kv_device_pool_limit(uint64_t bytes);
int kv_device_trim(int device);
/* phase i of the kv_validate that produced r: its name ("upload", "setup", "pass", "host_alloc",
 * "status_d2h", "records_count", "records_scatter_d2h", ...) and wall-clock milliseconds;
 * KV_E_RANGE past the last phase. Diagnostics of the host boundary (no reference counterpart). */
int kv_result_phase(const kv_result* r, uint32_t i, const char** name, double* ms);
/* counts[(scope * n_rules + rule) * 8 + status] (KV_MODE_SCOPES) */
int kv_result_scope_counts(const kv_result* r, const int64_t** counts, uint32_t* n_scopes);
/* failing path of a FAIL pair, e.g. "/spec/containers/0/image/" (needs KV_MODE_ERRORS);
 * returns the string length, or a negative code. */
int kv_result_path(const kv_result* r, uint32_t rule, uint64_t res, char* buf, size_t cap);
/* raw error record: kind (validate.go/anchor.go error form) and anchor-wrap flags */
int kv_result_error(const kv_result* r, uint32_t rule, uint64_t res, uint32_t* kind, uint32_t* flags);
/* err.Error() of the PatternError behind a FAIL / ERROR / SKIP pair — the SKIP
 * message and the "execution error: %s" operand of the ERROR message
 * (pkg/engine/validation.go:421-439,510-527; error forms of
 * pkg/engine/validate/validate.go:62-172 and pkg/engine/anchor/anchor.go:61-261).
 * The caller passes the resource document (JSON) it ingested, from which the
 * Go '%v' / %T operands are formatted. Returns the message length, KV_E_INVALID
 * for other statuses or constant (compile-time) statuses, KV_E_PARSE for bad JSON. */
int kv_result_error_message(const kv_result* r, uint32_t rule, uint64_t res, const char* resource_json, size_t len,
                            char* buf, size_t cap);

/* Pattern variables: when rule `rule` is ERROR on `res` because
 * substituting the `{{request.object...}}` variables of its pattern failed, writes the
 * RuleResponse message "variable substitution failed: <error>" (pkg/engine/validation.go:
 * 181-189, the reference's processValidationRule -> substitutePatterns) and returns its
 * length; 0 when the pair's status has another cause. */
int kv_result_subst_error(const kv_result* r, uint32_t rule, uint64_t res, char* buf, size_t cap);
double kv_result_kernel_ms(const kv_result* r);

/* Bulk export of the failing pairs (KV_MODE_ERRORS): every FAIL / ERROR / SKIP pair,
 * rule-major and in resource order: pair i = (rule[i], res[i]); path_id[i] names the
 * failing path of a FAIL pair (KV_PATH_NONE for ERROR / SKIP), rendered once per
 * distinct path by kv_path_string (e.g. "/spec/containers/0/image/"; ids numbered by first
 * appearance in the returned order). The arrays and
 * strings live as long as the result. This is what a Go caller builds
 * RuleResponse.Message from without one call per pair (validation.go:510-547). */
enum { KV_PATH_NONE = 0xFFFFFFFFu };
int kv_result_failures(const kv_result* r, uint64_t* n, const uint32_t** rule, const uint64_t** res,
                       const uint32_t** path_id);
const char* kv_path_string(const kv_result* r, uint32_t path_id);

/* Benchmark entry: device-resident inputs, `iters` timed launches on one stream
 * bracketed by HIP events. Returns mean kernel milliseconds per pass over all
 * rules of the batch. */
int kv_bench(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, int device, uint32_t mode, int warmup,
             int iters, double* ms_per_iter, kv_error** err);

/* Session: device-resident inputs and output buffers allocated once
 * (kv_session_create, untimed); kv_session_run enqueues `iters` passes on the
 * session's stream and waits for them, returning the HIP-event time of the
 * passes (ms, total). For benchmarks and repeated background scans. */
typedef struct kv_session kv_session;
int kv_session_create(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, int device, uint32_t mode,
                      kv_session** out, kv_error** err);
/* multi-device session (see kv_validate_devices); kv_session_counts / _scope_counts
 * return the RCCL-reduced totals, kv_session_fetch the last pass as a result */
int kv_session_create_devices(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, uint32_t device_mask,
                              uint32_t mode, kv_session** out, kv_error** err);
int kv_session_parts(const kv_session* s, uint32_t* n_parts);
int kv_session_fetch(kv_session* s, kv_result** out, kv_error** err);
int kv_session_run(kv_session* s, int iters, double* event_ms, kv_error** err);
int kv_session_counts(kv_session* s, int64_t* counts /* [n_rules][8], last pass */);
int kv_session_scope_counts(kv_session* s, int64_t* counts /* [n_scopes][n_rules][8], last pass */);
void kv_free_session(kv_session* s);
/* Multi-device session assembled from per-device batches: each part's resources are
 * ingested on their own (a background-scan worker per GPU, or one host feeding G devices
 * without holding the whole node's batch; pkg/policy/policy_controller.go:453-454 ->
 * pkg/policy/apply.go:72). kv_session_create_parts opens a session of n_parts parts;
 * kv_session_attach_part uploads batch b to HIP device `device` as part `part` — the
 * session keeps only the device copy, so the caller may free b right after. When the last
 * part is attached the scopes become the sorted union of the parts' namespaces
 * (kv_session_scopes / kv_session_scope_name) and the RCCL communicator is created (distinct
 * devices); run / counts / scope_counts then work as for kv_session_create_devices
 * (KV_E_DEVICE before that). kv_session_fetch is not available (no host batch). */
int kv_session_create_parts(const kv_policyset* ps, const char* ctx_json, uint32_t mode, uint32_t n_parts,
                            kv_session** out, kv_error** err);
int kv_session_attach_part(kv_session* s, uint32_t part, const kv_batch* b, int device, kv_error** err);
/* scope table of a session (batch namespaces; the union of the parts' for a parts session) */
int kv_session_scopes(const kv_session* s, uint32_t* n_scopes);
const char* kv_session_scope_name(const kv_session* s, uint32_t i);
/* ranks of the session's RCCL communicator (0: counts summed on the host — one part, or
 * logical parts of one device) and the HIP-event ms of each part's last kv_session_run */
int kv_session_rccl_ranks(const kv_session* s, int* ranks);
int kv_session_part_ms(const kv_session* s, double* ms /* [n_parts] */);
/* status-matrix bytes the last pass wrote: the specialized kernels write a rule's statuses of a
 * 256-resource workgroup only when one of them is not NOMATCH and flag the segment (an unwritten
 * segment is filled with NOMATCH at fetch); the bytecode engine writes the whole matrix. The
 * output bytes of a pass for the roofline accounting (no reference counterpart). */
int kv_session_status_bytes(kv_session* s, uint64_t* bytes);

/* Synthetic resource generator for the benchmark configs:
 * kind_mix 0 = Pods; 1 = Pods/Deployments/Services 60/25/15 (64 namespaces each);
 * 2 = the mixed kinds over 1 000 namespaces (C3). Returns NDJSON
 * (free with kv_free_buffer). */
int kv_synth(uint64_t seed, uint64_t n, uint32_t kind_mix, char** json_out, size_t* len);
/* resources [first, first + n) of the same stream (a rank's contiguous shard) */
int kv_synth_range(uint64_t seed, uint64_t first, uint64_t n, uint32_t kind_mix, char** json_out, size_t* len);

void kv_free_policyset(kv_policyset* ps);
void kv_free_batch(kv_batch* b);
void kv_free_result(kv_result* r);
void kv_free_error(kv_error* e);
void kv_free_buffer(char* p);

#ifdef __cplusplus
}
#endif
#endif /* KVGPU_H */
