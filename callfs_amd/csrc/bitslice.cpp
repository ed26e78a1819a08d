// Runtime of the bit-sliced kernels (bitslice.hpp): hiprtc compile, code-object cache,
// per-device modules, the background compile worker and the launch.
#include "bitslice.hpp"

#include <hip/hip_ext.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <sstream>
#include <thread>
#include <sys/stat.h>
#include <unistd.h>
#include <cstddef>

namespace callfs {
namespace bs {

static_assert(sizeof(Args) == 56 && offsetof(Args, nvec) == 24 && offsetof(Args, order) == 52,
              "Args: the layout args_decl() declares to the generated source");

namespace {

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

// gfx950 (or the device's own gfx name when one is current); CALLFS_OFFLOAD_ARCH overrides.
// Resolved on the thread that creates the kernel (kernel_for), never on the compile worker:
// the worker makes no HIP call, so one still compiling at process exit cannot race the HIP
// runtime's teardown.
std::string device_arch() {
  // only a well-formed target name (gfx + 3 or 4 hex digits: gfx90a, gfx950, gfx1201): hiprtc
  // on a GPU box crashed on "gfx1" instead of failing the compile
  if (const char* e = std::getenv("CALLFS_OFFLOAD_ARCH")) {
    const std::string a = e;
    bool ok = (a.size() == 6 || a.size() == 7) && a.compare(0, 3, "gfx") == 0;
    for (size_t i = 3; ok && i < a.size(); ++i) ok = std::isxdigit(static_cast<unsigned char>(a[i])) != 0;
    if (ok) return a;
  }
  int dev = -1;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) {
    std::string a = p.gcnArchName;
    const size_t colon = a.find(':');
    if (colon != std::string::npos) a.resize(colon);
    if (!a.empty()) return a;
  }
  return "gfx950";
}
std::string target_arch() {
  static const std::string a = device_arch();  // once per process (one gfx target per box)
  return a;
}

// On-disk cache of code objects: CALLFS_RS_JIT_CACHE (a directory; "0" turns it off), else
// $XDG_CACHE_HOME/callfs_rs or $HOME/.cache/callfs_rs. Files are written whole and renamed
// into place, so concurrent processes never read a partial one.
std::string cache_dir() {
  const char* e = std::getenv("CALLFS_RS_JIT_CACHE");
  if (e) return std::strcmp(e, "0") == 0 ? std::string() : std::string(e);
  if (const char* x = std::getenv("XDG_CACHE_HOME")) return std::string(x) + "/callfs_rs";
  if (const char* h = std::getenv("HOME")) return std::string(h) + "/.cache/callfs_rs";
  return std::string();
}

// A cache entry: a 16-B header ("CFBS", the waves-per-SIMD floor the search settled on, the
// spilled VGPRs, the code object's size) and the code object. An entry that does not parse,
// whose size disagrees or whose code is not an ELF object is a miss (then recompiled).
constexpr char kCacheMagic[4] = {'C', 'F', 'B', 'S'};

bool read_entry(const std::string& path, std::vector<char>& code, int* waves, int* spills) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::vector<char> all((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (all.size() <= 16 || std::memcmp(all.data(), kCacheMagic, 4) != 0) return false;
  int32_t hdr[3];
  std::memcpy(hdr, all.data() + 4, sizeof hdr);
  if (hdr[2] <= 0 || static_cast<size_t>(hdr[2]) != all.size() - 16) return false;
  if (std::memcmp(all.data() + 16, "\x7f" "ELF", 4) != 0) return false;
  code.assign(all.begin() + 16, all.end());
  *waves = hdr[0];
  *spills = hdr[1];
  return true;
}

void write_entry(const std::string& dir, const std::string& path, const std::vector<char>& code,
                 int waves, int spills) {
  if (dir.empty()) return;
  // mkdir -p of the cache directory
  std::string acc;
  std::stringstream ss(dir);
  std::string part;
  if (dir[0] == '/') acc = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    acc += part + "/";
    (void)::mkdir(acc.c_str(), 0755);
  }
  const std::string tmp = path + ".tmp." + std::to_string(::getpid());
  const int32_t hdr[3] = {waves, spills, static_cast<int32_t>(code.size())};
  bool ok;
  {
    std::ofstream f(tmp, std::ios::binary);
    f.write(kCacheMagic, 4);
    f.write(reinterpret_cast<const char*>(hdr), sizeof hdr);
    f.write(code.data(), static_cast<std::streamsize>(code.size()));
    f.close();
    ok = static_cast<bool>(f);
  }
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) (void)std::remove(tmp.c_str());
}

}  // namespace

// One background thread compiles queued kernels in order.
//
// Exit: the process's static destructors include hiprtc / comgr's, some of them registered
// during the first compile. A compile still running on the worker while they run used freed
// comgr memory (SIGSEGV or a double free at exit, tests/native/bs_worker.cpp), so the worker
// is never destroyed; instead the first push compiles a small kernel (comgr's lazy state now
// exists) and then registers drain() with atexit. Handlers run in reverse order of
// registration, so drain() -- drop the queue, let the compile in flight finish, join --
// runs before comgr's destructors.
class Worker {
 public:
  static Worker& get() {
    static Worker* w = new Worker;  // never destroyed (see above)
    return *w;
  }
  void push(const std::shared_ptr<Kernel>& k) {
    std::call_once(init_, [] {
      warm_compiler();
      std::atexit([] { Worker::get().drain(); });
    });
    std::lock_guard<std::mutex> g(mu_);
    // exiting, or a fork's child (the thread is the parent's): the kernel stays queued and
    // launches keep the nibble tables
    if (stop_ || (th_.joinable() && owner_ != ::getpid())) return;
    if (!th_.joinable()) {
      th_ = std::thread([this] { loop(); });
      owner_ = ::getpid();
    }
    q_.push_back(k);
    cv_.notify_one();
  }
  void drain() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      q_.clear();
    }
    cv_.notify_all();
    // a fork's child exits without the parent's thread (never joined: the Worker is immortal)
    if (th_.joinable() && owner_ == ::getpid()) th_.join();
  }

 private:
  static void warm_compiler();
  void loop() {
    for (;;) {
      std::shared_ptr<Kernel> k;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (stop_) return;
        k = q_.front().lock();
        q_.pop_front();
      }
      if (k) k->compile_now();
    }
  }
  std::once_flag init_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::weak_ptr<Kernel>> q_;
  std::thread th_;
  pid_t owner_ = 0;  // the process that started th_
  bool stop_ = false;
};

Mode mode() {
  static const Mode m = [] {
    const char* e = std::getenv("CALLFS_RS_BITSLICE");
    if (!e || !*e) return Mode::kAuto;
    if (!std::strcmp(e, "0") || !std::strcmp(e, "off")) return Mode::kOff;
    if (!std::strcmp(e, "sync")) return Mode::kSync;
    return Mode::kAuto;
  }();
  return m;
}

Kernel::Kernel(int K, int R, const uint8_t* coef)
    : net_(build_network(K, R, coef)), arch_(target_arch()) {
  (void)R;
  opt_.prefetch = 0;   // auto at compile time (compile_locked)
  opt_.min_waves = 0;  // auto_waves at compile time
  // development knobs (tools/bs_probe.py): prefetch depth and the waves-per-SIMD floor
  if (const char* e = std::getenv("CALLFS_RS_BS_PREFETCH")) opt_.prefetch = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("CALLFS_RS_BS_WAVES")) opt_.min_waves = std::max(1, std::min(8, std::atoi(e)));
  if (const char* e = std::getenv("CALLFS_RS_BS_BLOCK")) {
    const int b = std::atoi(e);
    if (b == 64 || b == 128 || b == 256 || b == 512 || b == 1024) opt_.block = b;
  }
}

Kernel::~Kernel() {
  for (int d = 0; d < kMaxDevices; ++d)
    if (mod_[d]) (void)hipModuleUnload(mod_[d]);
}

Kernel::State Kernel::state() const {
  std::lock_guard<std::mutex> g(mu_);
  return state_;
}

void Kernel::compile_async() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (state_ != State::kIdle) return;
    state_ = State::kQueued;
  }
  Worker::get().push(shared_from_this());
}

bool Kernel::compile_now() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    if (state_ == State::kReady) return true;
    if (state_ == State::kFailed) return false;
    if (state_ == State::kCompiling) {
      cv_.wait(lk);
      continue;
    }
    compile_locked(lk);
  }
}

namespace {
// One hiprtc compile of `src`; the code object, or empty with *err set. *spills = the
// compiler's "VGPRs Spill" remark for the kernel (-1 when the log has none).
std::vector<char> rtc_compile(const std::string& src, const std::vector<std::string>& opts,
                              std::string* err, int* spills) {
  std::vector<char> code;
  *spills = -1;
  hiprtcProgram p = nullptr;
  if (hiprtcCreateProgram(&p, src.c_str(), "rs_bs.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    *err = "hiprtcCreateProgram failed";
    return code;
  }
  std::vector<const char*> o;
  for (const auto& x : opts) o.push_back(x.c_str());
  const hiprtcResult r = hiprtcCompileProgram(p, static_cast<int>(o.size()), o.data());
  size_t n = 0;
  (void)hiprtcGetProgramLogSize(p, &n);
  std::string log(n, '\0');
  if (n) (void)hiprtcGetProgramLog(p, &log[0]);
  const size_t at = log.find("VGPRs Spill:");
  if (at != std::string::npos) *spills = std::atoi(log.c_str() + at + 12);
  if (r != HIPRTC_SUCCESS) {
    *err = std::string("hiprtc: ") + hiprtcGetErrorString(r) + "\n" + log;
  } else {
    if (hiprtcGetCodeSize(p, &n) == HIPRTC_SUCCESS && n) {
      code.resize(n);
      if (hiprtcGetCode(p, code.data()) != HIPRTC_SUCCESS) code.clear();
    }
    if (code.empty()) *err = "hiprtc: no code object";
  }
  (void)hiprtcDestroyProgram(&p);
  return code;
}

// Waves per SIMD to ask for: the VGPRs a group needs are about 8 accumulator planes per row,
// 8 per input shard in flight and ~40 for the planes and combos of the shard being consumed
// and addresses; 512 VGPRs per SIMD lane (tools/jobs.sh bs_params_r06, profiles/r06/params1: R = 8
// at 4 waves 75.9 -> 79.1 % for RS(32,8) 2 MiB; R = 16 forced to 3 waves spilled ~1,000 VGPRs
// and ran at 12 %).
int auto_waves(int R, int prefetch) {
  const int need = 8 * R + 8 * (prefetch + 1) + 40;
  return std::max(1, std::min(8, 512 / need));
}
constexpr int kSpillLimit = 16;  // VGPRs spilled that a floor may cost before it is lowered
}  // namespace

void Worker::warm_compiler() {
  // the constructs the generated kernels use (a bit-select, non-temporal 16-B loads and stores)
  static const char* src =
      "typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));\n"
      "extern \"C\" __global__ void warm(const u32x4* a, u32x4* b) {\n"
      "  u32x4 x = __builtin_nontemporal_load(a + threadIdx.x);\n"
      "  x.x = __builtin_amdgcn_bitop3_b32(x.x, x.y, x.z, 0xCA);\n"
      "  __builtin_nontemporal_store(x, b + threadIdx.x);\n"
      "}\n";
  std::string err;
  int spills = 0;
  (void)rtc_compile(src, {"--offload-arch=" + target_arch(), "-O3", "-std=c++17", "-fno-gpu-rdc"},
                    &err, &spills);
}

void Kernel::compile_locked(std::unique_lock<std::mutex>& lk) {
  state_ = State::kCompiling;
  const Network net = net_;
  GenOptions opt = opt_;
  lk.unlock();
  const auto t0 = std::chrono::steady_clock::now();
  const std::string arch = arch_;
  // two shards in flight; groups that run at 2 waves per SIMD anyway have the registers for
  // four (profiles/r06/params1: RS(32,16) 74.8 -> 75.3 %, RS(20,16) 256 KiB 74.8 -> 75.3 %)
  if (opt.prefetch <= 0) opt.prefetch = auto_waves(net.R, 2) <= 2 ? 4 : 2;
  if (opt.min_waves <= 0) opt.min_waves = auto_waves(net.R, opt.prefetch);
  std::string src = kernel_source(net, "rs_bs", opt, sizeof(Args));
  int ver_major = 0, ver_minor = 0;
  (void)hiprtcVersion(&ver_major, &ver_minor);
  const std::vector<std::string> opts = {"--offload-arch=" + arch, "-O3", "-std=c++17",
                                         "-fno-gpu-rdc", "-Rpass-analysis=kernel-resource-usage"};
  // keyed by the first source tried: the cache holds the code object the search accepted
  std::string keytxt = src + arch + std::to_string(ver_major) + "." + std::to_string(ver_minor);
  for (const auto& o : opts) keytxt += o;
  char name[64];
  std::snprintf(name, sizeof name, "bs-%016llx.co", static_cast<unsigned long long>(fnv1a(keytxt)));
  const std::string dir = cache_dir();
  const std::string path = dir.empty() ? std::string() : dir + "/" + name;
  std::vector<char> code;
  std::string err;
  int spills = -1;
  int cached_waves = 0;
  if (!path.empty() && read_entry(path, code, &cached_waves, &spills)) {
    opt.min_waves = cached_waves;
  } else {
    code.clear();
    spills = -1;
    // lower the waves-per-SIMD floor while the compiler spills more than kSpillLimit VGPRs
    for (;;) {
      code = rtc_compile(src, opts, &err, &spills);
      if (code.empty() || spills <= kSpillLimit || opt.min_waves <= 1) break;
      --opt.min_waves;
      src = kernel_source(net, "rs_bs", opt, sizeof(Args));
    }
    if (!code.empty() && !path.empty()) write_entry(dir, path, code, opt.min_waves, spills);
  }
  const double secs =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  lk.lock();
  compile_s_ = secs;
  spills_ = spills;
  waves_ = opt.min_waves;
  if (code.empty()) {
    error_ = err;
    state_ = State::kFailed;
    if (std::getenv("CALLFS_RS_BITSLICE_LOG"))
      std::fprintf(stderr, "callfs_rs bitslice K=%d R=%d: %s\n", net.K, net.R, err.c_str());
  } else {
    code_ = std::move(code);
    state_ = State::kReady;
    if (std::getenv("CALLFS_RS_BITSLICE_LOG"))
      std::fprintf(stderr, "callfs_rs bitslice K=%d R=%d: %zu B code object, %d waves floor, "
                   "%d VGPRs spilled, %.2f s\n", net.K, net.R, code_.size(), waves_, spills, secs);
  }
  cv_.notify_all();
}

hipFunction_t Kernel::function(int device, bool wait) {
  if (device < 0 || device >= kMaxDevices) return nullptr;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (fn_[device]) return fn_[device];
  }
  if (wait) {
    if (!compile_now()) return nullptr;
  } else if (state() != State::kReady) {
    compile_async();
    return nullptr;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (fn_[device]) return fn_[device];
  if (state_ != State::kReady) return nullptr;
  hipModule_t m = nullptr;
  hipFunction_t f = nullptr;
  if (hipModuleLoadData(&m, code_.data()) != hipSuccess) return nullptr;
  if (hipModuleGetFunction(&f, m, "rs_bs") != hipSuccess) {
    (void)hipModuleUnload(m);
    return nullptr;
  }
  int regs = 0;
  if (hipFuncGetAttribute(&regs, HIP_FUNC_ATTRIBUTE_NUM_REGS, f) == hipSuccess) vgprs_ = regs;
  mod_[device] = m;
  fn_[device] = f;
  return f;
}

std::shared_ptr<Kernel> kernel_for(int K, int R, const uint8_t* coef) {
  // never destroyed: modules stay loaded until the process ends (unloading them from a
  // static destructor could run after the HIP runtime's own teardown)
  static auto* mu = new std::mutex;
  static auto* map = new std::map<std::string, std::shared_ptr<Kernel>>;
  std::string key(reinterpret_cast<const char*>(&K), sizeof K);
  key.append(reinterpret_cast<const char*>(&R), sizeof R);
  key.append(reinterpret_cast<const char*>(coef), static_cast<size_t>(K) * R);
  std::lock_guard<std::mutex> g(*mu);
  auto it = map->find(key);
  if (it != map->end()) return it->second;
  // bounded like the coefficient-table cache (rs_capi.cpp TableCache): past kCap entries the
  // kernels no table set or compile holds any more are dropped (their modules unloaded)
  constexpr size_t kCap = 1024;
  if (map->size() >= kCap)
    for (auto i = map->begin(); i != map->end();) i = i->second.use_count() == 1 ? map->erase(i) : std::next(i);
  auto k = std::make_shared<Kernel>(K, R, coef);
  map->emplace(key, k);
  return k;
}

hipError_t launch(hipFunction_t fn, const Args& a, uint32_t tiles, int block, hipStream_t stream,
                  hipEvent_t ev_start, hipEvent_t ev_stop) {
  Args args = a;
  size_t size = sizeof args;
  void* config[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                    HIP_LAUNCH_PARAM_END};
  if (ev_start || ev_stop)
    return hipExtModuleLaunchKernel(fn, tiles * static_cast<uint32_t>(block), 1, 1,
                                    static_cast<uint32_t>(block), 1, 1, 0, stream, nullptr, config,
                                    ev_start, ev_stop, 0);
  return hipModuleLaunchKernel(fn, tiles, 1, 1, static_cast<uint32_t>(block), 1, 1, 0, stream,
                               nullptr, config);
}

}  // namespace bs
}  // namespace callfs
