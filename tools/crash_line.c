/* crash_line.c — bench.py's last-words hook (tools/lib/libcrashline.so).
 *
 * bench.py's N > 1 run measures the main schedule first and then a list of
 * comparison schedules before it prints its one JSON line. If a comparison
 * ends the process instead of returning an error (a GPU fault is SIGABRT from
 * the HIP runtime; torchrun stops the surviving ranks with SIGTERM when one
 * rank dies), the line measured so far would be lost with it. bench.py hands
 * that line to this hook; on a fatal signal the handler writes it to stdout
 * (write(2) is async-signal-safe), restores the default action and re-raises,
 * so the exit status still reports the signal.
 *
 * Not part of the product library: nothing under tips_amd/ loads it.
 */
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static char* volatile g_line = NULL; /* NUL-terminated, ends with '\n' */
static volatile sig_atomic_t g_fired = 0;

static void on_fatal(int sig) {
  char* line = g_line;
  if (line && !g_fired) {
    g_fired = 1;
    size_t len = strlen(line), off = 0;
    while (off < len) {
      ssize_t w = write(1, line + off, len - off);
      if (w <= 0) break;
      off += (size_t)w;
    }
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

/* Replace the line (a copy is kept; NULL or "" clears it). Returns 0, or -1 on allocation failure. */
int crash_line_set(const char* text) {
  char* fresh = NULL;
  if (text && *text) {
    size_t len = strlen(text);
    fresh = (char*)malloc(len + 2);
    if (!fresh) return -1;
    memcpy(fresh, text, len);
    fresh[len] = '\n';
    fresh[len + 1] = '\0';
  }
  /* the old buffer is leaked on purpose: a handler running on another thread may still read it */
  g_line = fresh;
  return 0;
}

/* Install the handler for the signals that end a process without Python unwinding. */
int crash_line_install(void) {
  static const int sigs[] = {SIGABRT, SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGTERM};
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_fatal;
  sigemptyset(&sa.sa_mask);
  for (size_t i = 0; i < sizeof sigs / sizeof sigs[0]; i++)
    if (sigaction(sigs[i], &sa, NULL) != 0) return -1;
  return 0;
}
