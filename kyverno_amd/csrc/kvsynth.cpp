// Deterministic synthetic Kubernetes resources for the benchmark configs
// (SURVEY.md §8d distributions). Output is NDJSON that goes through the normal
// kv_ingest path, exactly like resources loaded from files.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>

#include "../../include/kvgpu.h"

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double u() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t n(uint32_t k) { return (uint32_t)(next() % k); }
};

const char* kRegistries[] = {"docker.io/", "gcr.io/", "quay.io/", "registry.local:5000/", ""};
const char* kPull[] = {"Always", "IfNotPresent", "Never"};
const char* kCpu[] = {"100m", "250m", "500m", "1", "2"};
const char* kCpu2[] = {"200m", "500m", "1", "2", "4"};
const char* kMem[] = {"64Mi", "128Mi", "256Mi", "512Mi", "1Gi", "2Gi"};
const char* kMem2[] = {"128Mi", "256Mi", "512Mi", "1Gi", "2Gi", "4Gi"};
const char* kApps[] = {"web", "api", "db", "cache", "worker", "frontend", "backend", "batch"};
const char* kOwners[] = {"team-a", "team-b", "team-c", "platform"};
const char* kTiers[] = {"frontend", "backend", "data"};
const char* kSeccomp[] = {"RuntimeDefault", "Localhost", "Unconfined"};
const char* kCaps[] = {"NET_ADMIN", "SYS_TIME", "CHOWN", "NET_BIND_SERVICE"};

void repo_name(std::string& o, uint32_t k) {
  static const char* a[] = {"nginx", "redis", "postgres", "busybox", "alpine", "envoy", "app", "svc",
                            "mysql", "mongo", "kafka", "zookeeper", "etcd", "coredns", "proxy", "agent"};
  o += a[k % 16];
  o += "-";
  o += std::to_string(k / 16);
}

void image(std::string& o, Rng& r) {
  o += kRegistries[r.n(5)];
  repo_name(o, r.n(256));
  double t = r.u();
  if (t < 0.15) {
    o += ":latest";
  } else if (t < 0.75) {
    o += ":v" + std::to_string(r.n(4)) + "." + std::to_string(r.n(20)) + "." + std::to_string(r.n(10));
  } else if (t < 0.85) {
    o += "@sha256:";
    static const char* hx = "0123456789abcdef";
    for (int i = 0; i < 64; i++) o.push_back(hx[r.n(16)]);
  }
}

void container(std::string& o, Rng& r, int idx, bool init) {
  o += "{\"name\":\"";
  o += init ? "init" : "c";
  o += std::to_string(idx) + "\",\"image\":\"";
  image(o, r);
  o += "\"";
  uint32_t pp = r.n(4);
  if (pp < 3) { o += ",\"imagePullPolicy\":\""; o += kPull[pp]; o += "\""; }
  if (r.u() < 0.7) {
    uint32_t c = r.n(5), m = r.n(6);
    double form = r.u();
    std::string cpu = std::string("\"") + kCpu[c] + "\"";
    if (form < 0.05) cpu = "1";
    else if (form < 0.08) cpu = "0.5";
    o += ",\"resources\":{\"requests\":{\"cpu\":" + cpu + ",\"memory\":\"" + kMem[m] + "\"},\"limits\":{\"cpu\":\"" +
         kCpu2[c] + "\",\"memory\":\"" + kMem2[m] + "\"}}";
  }
  if (r.u() < 0.8) {
    o += ",\"securityContext\":{";
    bool first = true;
    auto field = [&](const std::string& f) {
      if (!first) o += ",";
      first = false;
      o += f;
    };
    if (r.u() < 0.6) field(std::string("\"privileged\":") + (r.u() < 0.1 ? "true" : "false"));
    if (r.u() < 0.6) field(std::string("\"runAsNonRoot\":") + (r.u() < 0.8 ? "true" : "false"));
    if (r.u() < 0.4) field("\"runAsGroup\":" + std::to_string(r.n(3) * 1000));
    if (r.u() < 0.6) field(std::string("\"allowPrivilegeEscalation\":") + (r.u() < 0.2 ? "true" : "false"));
    if (r.u() < 0.1) field(std::string("\"capabilities\":{\"add\":[\"") + kCaps[r.n(4)] + "\"]}");
    if (r.u() < 0.5) field(std::string("\"seccompProfile\":{\"type\":\"") + kSeccomp[r.n(3)] + "\"}");
    if (r.u() < 0.05) field(std::string("\"procMount\":\"") + (r.u() < 0.5 ? "Default" : "Unmasked") + "\"");
    if (r.u() < 0.03) field("\"seLinuxOptions\":{\"type\":\"spc_t\"}");
    o += "}";
  }
  if (r.u() < 0.6) {
    o += ",\"ports\":[{\"containerPort\":" + std::to_string(8000 + r.n(100));
    if (r.u() < 0.05) o += ",\"hostPort\":" + std::to_string(30000 + r.n(1000));
    o += "}]";
  }
  o += "}";
}

void pod_spec(std::string& o, Rng& r) {
  o += "{";
  double ic = r.u();
  if (ic >= 0.8) {
    o += "\"initContainers\":[";
    container(o, r, 0, true);
    o += "],";
  }
  double cc = r.u();
  int n = cc < 0.5 ? 1 : cc < 0.8 ? 2 : cc < 0.95 ? 3 : 4;
  o += "\"containers\":[";
  for (int i = 0; i < n; i++) {
    if (i) o += ",";
    container(o, r, i, false);
  }
  o += "]";
  if (r.u() < 0.05) o += ",\"hostNetwork\":true";
  if (r.u() < 0.05) o += ",\"hostPID\":true";
  // pod-level fields for the anchor-heavy chart rules (configs C4/C5) come from a side stream
  // so the main stream (and every earlier workload) is unchanged
  Rng q{r.s ^ 0xC4C5A11CE5ull};
  std::string sc;
  auto scf = [&](const std::string& f) { sc += sc.empty() ? "" : ","; sc += f; };
  if (r.u() < 0.05) {
    std::string sy = "\"sysctls\":[{\"name\":\"";
    sy += r.u() < 0.5 ? "kernel.shm_rmid_forced" : "net.core.somaxconn";
    sy += "\",\"value\":\"1\"}]";
    scf(sy);
  }
  if (q.u() < 0.25) scf(std::string("\"runAsNonRoot\":") + (q.u() < 0.85 ? "true" : "false"));
  if (q.u() < 0.20) scf("\"runAsGroup\":" + std::to_string(q.u() < 0.1 ? 0 : 1000 + q.n(3) * 1000));
  if (q.u() < 0.20) scf("\"fsGroup\":" + std::to_string(q.u() < 0.1 ? 0 : 2000));
  if (q.u() < 0.10) scf(std::string("\"supplementalGroups\":[") + (q.u() < 0.2 ? "0" : "3000") + ",4000]");
  if (q.u() < 0.20) scf(std::string("\"seccompProfile\":{\"type\":\"") + kSeccomp[q.n(3)] + "\"}");
  if (!sc.empty()) o += ",\"securityContext\":{" + sc + "}";
  if (q.u() < 0.03) o += ",\"hostIPC\":true";
  double v = r.u();
  if (v < 0.05) o += ",\"volumes\":[{\"name\":\"host\",\"hostPath\":{\"path\":\"/var/run\"}}]";
  else if (v < 0.4) {
    // restricted volume types (restrict-volume-types) on a small share
    double t = q.u();
    if (t < 0.04) o += ",\"volumes\":[{\"name\":\"data\",\"nfs\":{\"server\":\"nfs\",\"path\":\"/x\"}}]";
    else if (t < 0.06) o += ",\"volumes\":[{\"name\":\"data\",\"csi\":{\"driver\":\"d\"}}]";
    else o += ",\"volumes\":[{\"name\":\"data\",\"emptyDir\":{}}]";
  }
  o += "}";
}

void labels(std::string& o, Rng& r) {
  o += "\"labels\":{";
  bool first = true;
  auto kv = [&](const char* k, const char* v) {
    if (!first) o += ",";
    first = false;
    o += std::string("\"") + k + "\":\"" + v + "\"";
  };
  if (r.u() < 0.9) kv("app", kApps[r.n(8)]);
  if (r.u() < 0.6) kv("owner", kOwners[r.n(4)]);
  if (r.u() < 0.5) kv("tier", kTiers[r.n(3)]);
  o += "}";
}

// n_ns namespaces "ns-0" .. "ns-<n_ns - 1>" (one draw either way, so the rest of a
// resource does not depend on n_ns)
void metadata(std::string& o, Rng& r, const char* prefix, uint64_t i, uint32_t n_ns) {
  o += "\"metadata\":{\"name\":\"";
  o += prefix;
  o += std::to_string(i) + "\",\"namespace\":\"ns-" + std::to_string(r.n(n_ns)) + "\",";
  labels(o, r);
  if (r.u() < 0.05) o += ",\"annotations\":{\"container.apparmor.security.beta.kubernetes.io/c0\":\"runtime/default\"}";
  o += "}";
}


// resource i of stream `seed`: its own generator state, so any contiguous range
// [first, first + n) of one stream is reproducible on its own (the shard of a rank).
// kind_mix 0: Pods, 64 namespaces (C2 / C4); 1: Pods/Deployments/Services 60/25/15,
// 64 namespaces (C5); 2: the same kinds over 1 000 namespaces (C3)
void resource(std::string& o, uint64_t seed, uint64_t i, uint32_t kind_mix) {
  Rng r{seed};
  r.s = r.next() ^ (i * 0xD1B54A32D192ED03ull);
  (void)r.next();
  const uint32_t n_ns = kind_mix == 2 ? 1000u : 64u;
  double k = kind_mix != 0 ? r.u() : 0.0;
  if (k < 0.60) {
    o += "{\"apiVersion\":\"v1\",\"kind\":\"Pod\",";
    metadata(o, r, "pod-", i, n_ns);
    o += ",\"spec\":";
    pod_spec(o, r);
    o += "}\n";
  } else if (k < 0.85) {
    o += "{\"apiVersion\":\"apps/v1\",\"kind\":\"Deployment\",";
    metadata(o, r, "deploy-", i, n_ns);
    o += ",\"spec\":{\"replicas\":" + std::to_string(1 + r.n(5)) + ",\"template\":{\"metadata\":{";
    labels(o, r);
    o += "},\"spec\":";
    pod_spec(o, r);
    o += "}}}\n";
  } else {
    static const char* st[] = {"ClusterIP", "NodePort", "LoadBalancer"};
    o += "{\"apiVersion\":\"v1\",\"kind\":\"Service\",";
    metadata(o, r, "svc-", i, n_ns);
    o += std::string(",\"spec\":{\"type\":\"") + st[r.n(3)] + "\",\"ports\":[{\"port\":" + std::to_string(80 + r.n(1000)) + "}]}}\n";
  }
}

}  // namespace

extern "C" int kv_synth_range(uint64_t seed, uint64_t first, uint64_t n, uint32_t kind_mix, char** json_out,
                              size_t* len) {
  if (!json_out || !len || kind_mix > 2) return KV_E_INVALID;
  const unsigned T = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(16, n / 4096));
  std::vector<std::string> parts(T);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; t++)
    th.emplace_back([&, t]() {
      const uint64_t b = n * t / T, e = n * (t + 1) / T;
      parts[t].reserve((e - b) * 900);
      for (uint64_t i = b; i < e; i++) resource(parts[t], seed, first + i, kind_mix);
    });
  for (auto& x : th) x.join();
  size_t total = 0;
  for (auto& p : parts) total += p.size();
  *json_out = (char*)malloc(total + 1);
  if (!*json_out) return KV_E_NOMEM;
  size_t at = 0;
  for (auto& p : parts) {
    memcpy(*json_out + at, p.data(), p.size());
    at += p.size();
  }
  (*json_out)[total] = 0;
  *len = total;
  return 0;
}

extern "C" int kv_synth(uint64_t seed, uint64_t n, uint32_t kind_mix, char** json_out, size_t* len) {
  return kv_synth_range(seed, 0, n, kind_mix, json_out, len);
}
