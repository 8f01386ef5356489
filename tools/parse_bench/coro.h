// Experiment: two pictures' parsers on one thread, switched at every residual
// block by a minimal stackful context switch (x86-64 SysV: callee-saved registers + rsp), so the
// core's out-of-order window holds the tail of one picture's CABAC chain and the head of the
// other's.  parse_bench -c pairs the pictures of its list; hevc_parser.cpp calls g_h2j_yield
// before each residual_coding when built with -DH2J_CORO.
#pragma once
#include <cstdint>
#include <cstdlib>

extern "C" void h2j_ctx_swap(void** save_sp, void* new_sp);
asm(R"(
.text
.globl h2j_ctx_swap
.type h2j_ctx_swap,@function
h2j_ctx_swap:
  pushq %rbp
  pushq %rbx
  pushq %r12
  pushq %r13
  pushq %r14
  pushq %r15
  movq %rsp, (%rdi)
  movq %rsi, %rsp
  popq %r15
  popq %r14
  popq %r13
  popq %r12
  popq %rbx
  popq %rbp
  ret
.size h2j_ctx_swap, .-h2j_ctx_swap
.globl h2j_ctx_boot
.type h2j_ctx_boot,@function
h2j_ctx_boot:
  movq %r12, %rdi
  callq *%r13
  ud2
.size h2j_ctx_boot, .-h2j_ctx_boot
)");
extern "C" void h2j_ctx_boot();

namespace h2j_coro {
struct Co {
    void* sp = nullptr;
    bool done = false;
    void* stack = nullptr;
};
// a fresh context that starts fn(arg) on its own stack (fn never returns)
inline void make(Co& c, size_t bytes, void (*fn)(void*), void* arg) {
    c.stack = std::malloc(bytes);
    uintptr_t top = (reinterpret_cast<uintptr_t>(c.stack) + bytes) & ~uintptr_t(15);
    uint64_t* s = reinterpret_cast<uint64_t*>(top);
    s[-1] = reinterpret_cast<uint64_t>(&h2j_ctx_boot);
    s[-2] = 0;                                    // rbp
    s[-3] = 0;                                    // rbx
    s[-4] = reinterpret_cast<uint64_t>(arg);      // r12
    s[-5] = reinterpret_cast<uint64_t>(fn);       // r13
    s[-6] = 0;                                    // r14
    s[-7] = 0;                                    // r15
    c.sp = s - 7;
}
}  // namespace h2j_coro
