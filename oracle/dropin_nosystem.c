/* oracle/dropin_nosystem.c — linked into the drop-in reference application only
 * (oracle/Makefile target `dropin`, with -Wl,--wrap=system).
 *
 * The reference main() converts each PPM with std::system("ffmpeg ...") and deletes it with
 * std::system("del ...") (RE/RaytracingEngine.cpp:313-322).  On the GPU box the process has
 * initialised the GPU by then, and a fork + exec of /bin/sh from such a process is refused or
 * unsafe.  With --wrap=system every such call lands here instead: nothing forks, the call
 * returns non-zero, and main() takes its own "conversion failed" branch — the PPMs it wrote
 * are kept, which is what tests/test_gpu_reference_app.py checks. */
#include <stdio.h>

int __wrap_system(const char* command) {
    fprintf(stderr, "[rtamd dropin] system() not run: %s\n", command ? command : "(null)");
    return command ? 1 : 0; /* system(NULL): "no command processor" */
}
