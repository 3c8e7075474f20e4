// rt_scene.h — host-side scene compiler interface (see rt_scene.cpp).
#pragma once
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_layout.h"

namespace rtl {

struct Compiled {
    SceneHdr hdr;
    std::vector<double> tab; // double table (offsets in hdr.o_*)
    std::vector<int> itab;   // int table (offsets in hdr.i_*)
};

int check_scene(const rt_elem *e, uint32_t n);
int fill_canon(rt_elem *e, uint32_t n);
int compile_scene(const rt_elem *e, uint32_t n, Compiled &out);

} // namespace rtl
