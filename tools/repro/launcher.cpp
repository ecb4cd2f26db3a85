// Loads the HIP runtime PyTorch-ROCm ships (HIP_RUNTIME_PATH, by full path, RTLD_GLOBAL) and then
// the reproducer library, whose libamdhip64.so.7 dependency the already-loaded runtime satisfies
// (the same binding libmp4x_hip.so gets inside a torch process); then runs it.  No HIP code here.
#include <dlfcn.h>
#include <cstdio>
#include <string>

int main(int argc, char** argv) {
  if (!dlopen(HIP_RUNTIME_PATH, RTLD_NOW | RTLD_GLOBAL)) {
    fprintf(stderr, "dlopen %s: %s\n", HIP_RUNTIME_PATH, dlerror());
    return 2;
  }
  std::string self = argv[0];
  const std::string dir = self.find('/') == std::string::npos ? "." : self.substr(0, self.rfind('/'));
  void* lib = dlopen((dir + "/libipc_lifetime_repro.so").c_str(), RTLD_NOW);
  if (!lib) {
    fprintf(stderr, "dlopen repro: %s\n", dlerror());
    return 2;
  }
  auto fn = reinterpret_cast<int (*)(int, char**)>(dlsym(lib, "repro_main"));
  if (!fn) {
    fprintf(stderr, "dlsym repro_main: %s\n", dlerror());
    return 2;
  }
  return fn(argc, argv);
}
