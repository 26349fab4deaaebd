/* segv_dump.c — diagnostic (not product): a SIGSEGV handler that prints the faulting address, the
 * interrupted PC and every backtrace frame as (library, offset, symbol) via dladdr, plus the library
 * mappings of /proc/self/maps, so a crash inside a tool or runtime library can be symbolized offline
 * (llvm-symbolizer --obj=<lib> <offset>).  Loaded with ctypes and installed after the profiler's own
 * handler (a later sigaction wins).  Build: gcc -shared -fPIC -O1 -o segv_dump.so segv_dump.c -ldl */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <ucontext.h>
#include <unistd.h>

static void frame(const char *tag, void *pc) {
  Dl_info info;
  memset(&info, 0, sizeof(info));
  if (dladdr(pc, &info) && info.dli_fname) {
    fprintf(stderr, "%s %p  %s+0x%lx  (%s)\n", tag, pc, info.dli_fname,
            (unsigned long)((char *)pc - (char *)info.dli_fbase), info.dli_sname ? info.dli_sname : "?");
  } else {
    fprintf(stderr, "%s %p  (no mapping)\n", tag, pc);
  }
}

static void handler(int sig, siginfo_t *si, void *ucv) {
  ucontext_t *uc = (ucontext_t *)ucv;
  void *pc = (void *)uc->uc_mcontext.gregs[REG_RIP];
  fprintf(stderr, "segv_dump: signal %d at address %p\n", sig, si->si_addr);
  frame("PC   ", pc);
  void *bt[96];
  int n = backtrace(bt, 96);
  for (int i = 0; i < n; i++) frame("frame", bt[i]);
  int fd = open("/proc/self/maps", O_RDONLY);
  if (fd >= 0) {
    char buf[65536];
    ssize_t k;
    fprintf(stderr, "segv_dump: maps (libraries, and the region around the fault)\n");
    while ((k = read(fd, buf, sizeof(buf) - 1)) > 0) {
      buf[k] = 0;
      char *line = buf, *nl;
      while ((nl = strchr(line, '\n'))) {
        *nl = 0;
        unsigned long a = 0, b = 0;
        sscanf(line, "%lx-%lx", &a, &b);
        unsigned long f = (unsigned long)si->si_addr;
        if (strstr(line, ".so") || (f >= a - (1ul << 24) && f < b + (1ul << 24))) fprintf(stderr, "%s\n", line);
        line = nl + 1;
      }
    }
    close(fd);
  }
  _exit(139);
}

void segv_dump_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO;
  sigaction(SIGSEGV, &sa, NULL);
  sigaction(SIGBUS, &sa, NULL);
}
