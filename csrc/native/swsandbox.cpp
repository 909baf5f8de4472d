// Script sandbox: a seccomp-BPF syscall allow-list for the isolated script worker process
// (sitewhere_amd/runtime/script_sandbox.py).
//
// Reference scripts (Groovy decoders, filters, routers -- GroovyComponent.java:25-166) run inside
// the JVM with full privileges.  Here an extension-point script can be run in a worker process that
// (1) sets resource limits, (2) pre-imports the modules scripts may use, then (3) calls
// sw_sandbox_lock(): after it, the process can only compute, allocate memory and talk over the pipes
// it already holds.  open/openat, socket/connect, execve, fork/clone, kill, ptrace, mount ... fail
// with EPERM, so an escape from the restricted Python namespace still cannot touch the host.
#include <errno.h>
#include <linux/audit.h>
#include <linux/filter.h>
#include <linux/seccomp.h>
#include <stddef.h>
#include <stdint.h>
#include <sys/prctl.h>
#include <sys/syscall.h>

#include <vector>

extern "C" {

// Returns 0 on success, -1 if the kernel refused (errno preserved), -2 on an unsupported arch.
int sw_sandbox_lock(void) {
#if defined(__x86_64__)
  const unsigned arch = AUDIT_ARCH_X86_64;
#elif defined(__aarch64__)
  const unsigned arch = AUDIT_ARCH_AARCH64;
#else
  return -2;
#endif
  static const int allowed[] = {
    SYS_read, SYS_write, SYS_readv, SYS_writev, SYS_close, SYS_lseek, SYS_fstat, SYS_newfstatat,
    SYS_mmap, SYS_munmap, SYS_mremap, SYS_mprotect, SYS_madvise, SYS_brk,
    SYS_rt_sigaction, SYS_rt_sigprocmask, SYS_rt_sigreturn, SYS_sigaltstack,
    SYS_futex, SYS_sched_yield, SYS_set_robust_list, SYS_rseq,
    SYS_clock_gettime, SYS_clock_getres, SYS_gettimeofday, SYS_clock_nanosleep, SYS_nanosleep,
    SYS_getpid, SYS_gettid, SYS_getrandom, SYS_getrusage, SYS_times,
    SYS_exit, SYS_exit_group,
#if defined(__x86_64__)
    SYS_poll, SYS_select,
#endif
    SYS_ppoll, SYS_pselect6,
  };
  const size_t n = sizeof(allowed) / sizeof(allowed[0]);
  std::vector<sock_filter> prog;
  // refuse a foreign syscall ABI outright (x32 / i386 entry points would bypass the numbers below)
  prog.push_back(BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, arch)));
  prog.push_back(BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, arch, 1, 0));
  prog.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_KILL_PROCESS));
  prog.push_back(BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, nr)));
  // prlimit64 only to read limits (new_limit == NULL): the worker's hard limits cannot be raised
  const unsigned a2 = (unsigned)(offsetof(struct seccomp_data, args) + 2 * sizeof(uint64_t));
  prog.push_back(BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, (unsigned)SYS_prlimit64, 0, 6));
  prog.push_back(BPF_STMT(BPF_LD | BPF_W | BPF_ABS, a2));                  // new_limit, low word
  prog.push_back(BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, 0, 0, 3));
  prog.push_back(BPF_STMT(BPF_LD | BPF_W | BPF_ABS, a2 + 4));              // high word
  prog.push_back(BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, 0, 0, 1));
  prog.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ALLOW));
  prog.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | (EPERM & SECCOMP_RET_DATA)));
  prog.push_back(BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(struct seccomp_data, nr)));
#if defined(__x86_64__)
  // x32 syscalls share the arch value with bit 30 set: deny them
  prog.push_back(BPF_JUMP(BPF_JMP | BPF_JGE | BPF_K, 0x40000000u, 0, 1));
  prog.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | (EPERM & SECCOMP_RET_DATA)));
#endif
  for (size_t i = 0; i < n; ++i) {
    // match -> fall through to ALLOW (at distance n - i), else test the next number
    prog.push_back(BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, (unsigned)allowed[i], (unsigned char)(n - i), 0));
  }
  prog.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | (EPERM & SECCOMP_RET_DATA)));
  prog.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ALLOW));
  sock_fprog fprog;
  fprog.len = (unsigned short)prog.size();
  fprog.filter = prog.data();
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0) return -1;
  if (prctl(PR_SET_SECCOMP, SECCOMP_MODE_FILTER, &fprog) != 0) return -1;
  return 0;
}

}  // extern "C"
