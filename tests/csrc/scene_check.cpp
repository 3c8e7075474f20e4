// Host-only sanitizer driver for the scene compiler (eraytracer_amd/csrc/rt_scene.cpp), built by
// tests/test_host.py with -fsanitize=address,undefined (GPU sanitizers are not available; the
// scene compiler is the library's host code that parses caller input).  Each argument is a file
// of rt_elem records exactly as the ctypes marshal lays them out; per file it prints
// "check canon compile n_tab n_itab".
#include <cstdio>
#include <vector>

#include "../../eraytracer_amd/csrc/rt_scene.h"

int main(int argc, char **argv) {
    for (int i = 1; i < argc; ++i) {
        FILE *f = std::fopen(argv[i], "rb");
        if (!f) return 2;
        std::vector<rt_elem> e;
        rt_elem x;
        while (std::fread(&x, sizeof x, 1, f) == 1) e.push_back(x);
        std::fclose(f);
        const uint32_t n = (uint32_t)e.size();
        const int rc_check = rtl::check_scene(e.data(), n);
        const int rc_canon = rtl::fill_canon(e.data(), n);
        rtl::Compiled c;
        const int rc_compile = rc_check == RT_OK ? rtl::compile_scene(e.data(), n, c) : rc_check;
        std::printf("%d %d %d %zu %zu\n", rc_check, rc_canon, rc_compile, c.tab.size(), c.itab.size());
    }
    return 0;
}
