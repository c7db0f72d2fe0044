// A fault report for the proxy-level load generator (tools/proxy_load.cpp):
// on SIGSEGV / SIGBUS it prints, to stderr,
//   - the fault address, whether the access was a read or a write (x86-64
//     page-fault error code), and the general registers (a memcpy's live
//     source / destination / count are in rsi / rdi / rcx);
//   - every frame of the faulting thread resolved with dladdr: the shared
//     object, its load base, the offset inside it and the nearest symbol;
//   - the lines of /proc/self/maps around the fault address and around the
//     memcpy pointers, so the buffer that ran out can be named;
// then restores the handler it replaced (the profiler's or Python's) and
// returns, so the faulting access repeats and that handler runs as before.
// Diagnostics only: nothing in the library installs signal handlers.  The
// text is formatted by hand into stack buffers and written with write(2)
// (no stdio, no allocation); backtrace() and dladdr() are not on POSIX's
// async-signal-safe list -- the unwinder is loaded at install() so the
// handler does not load it, and a fault taken while the dynamic loader's
// lock is held would hang the report, the cost every such reporter
// (glog's included) accepts.
#pragma once
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdint.h>
#include <string.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>

namespace crash_report {

inline struct sigaction g_old_segv, g_old_bus;
inline bool g_installed = false;

inline void say(const char* s) { (void)!write(2, s, strlen(s)); }

// Appends to a fixed buffer without stdio (Line::add / hex / dec).
struct Line {
  char b[1024];
  size_t n = 0;
  Line& add(const char* s) {
    while (*s && n + 1 < sizeof b) b[n++] = *s++;
    b[n] = 0;
    return *this;
  }
  Line& hex(uint64_t v, int digits = 0) {  // 0x-less; `digits` pads with zeros
    char t[17];
    int i = 16;
    t[i] = 0;
    do {
      t[--i] = "0123456789abcdef"[v & 15];
      v >>= 4;
    } while ((v || 16 - i < digits) && i > 0);
    return add(t + i);
  }
  Line& dec(int64_t v) {
    char t[24];
    int i = 23;
    t[i] = 0;
    const bool neg = v < 0;
    uint64_t u = neg ? 0 - (uint64_t)v : (uint64_t)v;
    do {
      t[--i] = (char)('0' + u % 10);
      u /= 10;
    } while (u && i > 1);
    if (neg) t[--i] = '-';
    return add(t + i);
  }
  void out() { say(b); }
};

inline void frame_line(const char* tag, void* pc) {
  Line l;
  l.add("  ").add(tag).add(" 0x").hex((uintptr_t)pc).add("  ");
  Dl_info di;
  if (dladdr(pc, &di) && di.dli_fname) {
    l.add(di.dli_fname).add("+0x").hex((uintptr_t)pc - (uintptr_t)di.dli_fbase);
    if (di.dli_sname) l.add("  (").add(di.dli_sname).add("+0x").hex((uintptr_t)pc - (uintptr_t)di.dli_saddr).add(")");
  } else {
    l.add("(no object)");
  }
  l.add("\n").out();
}

inline uintptr_t parse_hex(const char*& p) {
  uintptr_t v = 0;
  for (;; ++p) {
    const char c = *p;
    if (c >= '0' && c <= '9') v = v * 16 + (uintptr_t)(c - '0');
    else if (c >= 'a' && c <= 'f') v = v * 16 + (uintptr_t)(c - 'a' + 10);
    else break;
  }
  return v;
}

// Mapping lines within `window` bytes of any of the n addresses.
inline void maps_near(const uintptr_t* at, int n, uintptr_t window) {
  const int fd = open("/proc/self/maps", O_RDONLY);
  if (fd < 0) return;
  static char buf[1 << 16];
  char line[1024];
  size_t ll = 0;
  for (;;) {
    const ssize_t got = read(fd, buf, sizeof buf);
    if (got <= 0) break;
    for (ssize_t i = 0; i < got; ++i) {
      if (buf[i] != '\n') {
        if (ll + 1 < sizeof line) line[ll++] = buf[i];
        continue;
      }
      line[ll] = 0;
      const char* p = line;
      const uintptr_t lo = parse_hex(p);
      if (*p == '-') ++p;
      const uintptr_t hi = parse_hex(p);
      bool keep = false;
      for (int k = 0; k < n && !keep; ++k)
        keep = at[k] && at[k] + window >= lo && at[k] < hi + window;
      if (keep) {
        say("  map ");
        say(line);
        say("\n");
      }
      ll = 0;
    }
  }
  close(fd);
}

inline void on_fault(int sig, siginfo_t* si, void* ctx) {
  const ucontext_t* uc = (const ucontext_t*)ctx;
  const greg_t* g = uc->uc_mcontext.gregs;
  const uintptr_t addr = (uintptr_t)si->si_addr;
  const unsigned long err = (unsigned long)g[REG_ERR];
  Line h;
  h.add("\n=== proxy_load crash report: signal ").dec(sig).add(" code ").dec(si->si_code).add(" at 0x").hex(addr)
      .add(" (").add((err & 16) ? "instruction" : (err & 2) ? "write" : "read").add(" access, page-fault error 0x")
      .hex(err).add(") tid ").dec((int64_t)syscall(SYS_gettid)).add("\n");
  h.out();
  static const struct {
    const char* name;
    int reg;
  } regs[2][6] = {{{"rip", REG_RIP}, {"rsp", REG_RSP}, {"rdi", REG_RDI}, {"rsi", REG_RSI}, {"rdx", REG_RDX}, {"rcx", REG_RCX}},
                  {{"rax", REG_RAX}, {"rbx", REG_RBX}, {"r8 ", REG_R8}, {"r9 ", REG_R9}, {"r10", REG_R10}, {"r11", REG_R11}}};
  for (const auto& row : regs) {
    Line r;
    r.add(" ");
    for (const auto& x : row) r.add(" ").add(x.name).add(" ").hex((uint64_t)g[x.reg], 16);
    r.add("\n").out();
  }
  frame_line("pc   ", (void*)g[REG_RIP]);
  void* frames[64];
  const int nf = backtrace(frames, 64);
  for (int i = 0; i < nf; ++i) {
    Line t;
    t.add("#").dec(i);
    while (t.n < 5) t.add(" ");
    frame_line(t.b, frames[i]);
  }
  say("  mappings within 2 MiB of the fault address, rdi and rsi:\n");
  const uintptr_t at[3] = {addr, (uintptr_t)g[REG_RDI], (uintptr_t)g[REG_RSI]};
  maps_near(at, 3, (uintptr_t)2 << 20);
  say("=== end of crash report\n");
  // Hand the fault to the handler this one replaced: the access repeats.
  sigaction(SIGSEGV, &g_old_segv, nullptr);
  sigaction(SIGBUS, &g_old_bus, nullptr);
  (void)sig;
}

inline void install() {
  if (g_installed) return;
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  void* warm[2];
  (void)backtrace(warm, 2);  // loads the unwinder now, not inside the handler
  if (sigaction(SIGSEGV, &sa, &g_old_segv) == 0 && sigaction(SIGBUS, &sa, &g_old_bus) == 0) g_installed = true;
}

inline void uninstall() {
  if (!g_installed) return;
  sigaction(SIGSEGV, &g_old_segv, nullptr);
  sigaction(SIGBUS, &g_old_bus, nullptr);
  g_installed = false;
}

}  // namespace crash_report
