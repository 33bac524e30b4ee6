// kvjitc: compiles one specialized-kernel program with hiprtc for gfx950.
//
//   kvjitc <program.hip> <out.co> <name>
//
// libkvgpu spawns several of these (jit_compile, kvjit.cpp): hiprtc serialises
// compilations inside one process, so the kernel programs of a large policy set
// compile in parallel only across processes. The child never touches a GPU.
#include <hip/hiprtc.h>

#include <cstdio>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: kvjitc program.hip out.co name\n");
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    fprintf(stderr, "kvjitc: cannot read %s\n", argv[1]);
    return 2;
  }
  std::string src;
  char buf[1 << 16];
  for (size_t n; (n = fread(buf, 1, sizeof buf, f)) > 0;) src.append(buf, n);
  fclose(f);
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), (std::string(argv[3]) + ".hip").c_str(), 0, nullptr, nullptr) !=
      HIPRTC_SUCCESS) {
    fprintf(stderr, "kvjitc: hiprtcCreateProgram failed\n");
    return 1;
  }
  // the options of kvjit.cpp kOpts
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-label", "-Wno-unused-variable"};
  if (hiprtcCompileProgram(prog, (int)(sizeof opts / sizeof opts[0]), opts) != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    fprintf(stderr, "%s\n", log.substr(0, 4000).c_str());
    hiprtcDestroyProgram(&prog);
    return 1;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  std::vector<char> code(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  const std::string tmp = std::string(argv[2]) + ".part";
  FILE* o = fopen(tmp.c_str(), "wb");
  if (!o || fwrite(code.data(), 1, code.size(), o) != code.size()) {
    fprintf(stderr, "kvjitc: cannot write %s\n", argv[2]);
    return 1;
  }
  fclose(o);
  return rename(tmp.c_str(), argv[2]) == 0 ? 0 : 1;
}
