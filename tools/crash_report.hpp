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
// Diagnostics only: nothing in the library installs signal handlers.
#pragma once
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>

namespace crash_report {

inline struct sigaction g_old_segv, g_old_bus;
inline bool g_installed = false;

inline void say(const char* s) { (void)!write(2, s, strlen(s)); }

inline void frame_line(const char* tag, void* pc) {
  char buf[768];
  Dl_info di;
  if (dladdr(pc, &di) && di.dli_fname) {
    const uintptr_t off = (uintptr_t)pc - (uintptr_t)di.dli_fbase;
    if (di.dli_sname)
      snprintf(buf, sizeof buf, "  %s %p  %s+0x%lx  (%s+0x%lx)\n", tag, pc, di.dli_fname, (unsigned long)off,
               di.dli_sname, (unsigned long)((uintptr_t)pc - (uintptr_t)di.dli_saddr));
    else
      snprintf(buf, sizeof buf, "  %s %p  %s+0x%lx\n", tag, pc, di.dli_fname, (unsigned long)off);
  } else {
    snprintf(buf, sizeof buf, "  %s %p  (no object)\n", tag, pc);
  }
  say(buf);
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
  char buf[1024];
  snprintf(buf, sizeof buf,
           "\n=== proxy_load crash report: signal %d code %d at %p (%s access, page-fault error 0x%lx) tid %ld\n"
           "  rip %016llx rsp %016llx rdi %016llx rsi %016llx rdx %016llx rcx %016llx\n"
           "  rax %016llx rbx %016llx r8  %016llx r9  %016llx r10 %016llx r11 %016llx\n",
           sig, si->si_code, si->si_addr, (err & 16) ? "instruction" : (err & 2) ? "write" : "read", err,
           (long)syscall(SYS_gettid), (unsigned long long)g[REG_RIP], (unsigned long long)g[REG_RSP],
           (unsigned long long)g[REG_RDI], (unsigned long long)g[REG_RSI], (unsigned long long)g[REG_RDX],
           (unsigned long long)g[REG_RCX], (unsigned long long)g[REG_RAX], (unsigned long long)g[REG_RBX],
           (unsigned long long)g[REG_R8], (unsigned long long)g[REG_R9], (unsigned long long)g[REG_R10],
           (unsigned long long)g[REG_R11]);
  say(buf);
  frame_line("pc   ", (void*)g[REG_RIP]);
  void* frames[64];
  const int nf = backtrace(frames, 64);
  for (int i = 0; i < nf; ++i) {
    char tag[16];
    snprintf(tag, sizeof tag, "#%-4d", i);
    frame_line(tag, frames[i]);
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
