/* A deliberate heap overflow, built with the oracle's sanitizer flags: proves that the ASan runtime
 * preloaded into the child python catches a bad access inside a ctypes-loaded library (so a clean
 * sanitized oracle run means something).  Test infrastructure only. */
#include <stdlib.h>

int canary_overflow(int n) {
    int* a = (int*)malloc((size_t)n * sizeof(int));
    if (a == NULL) return -1;
    for (int i = 0; i < n; ++i) a[i] = i;
    int v = a[n];            /* one past the end */
    free(a);
    return v;
}
