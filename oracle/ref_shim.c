/*
 * ref_shim.c -- link-time instrumentation for building the REFERENCE programs
 * from their unmodified sources under /root/reference (oracle/Makefile).
 *
 * TEST INFRASTRUCTURE ONLY.  The reference drivers are linked with
 *   -Wl,--wrap=time -Wl,--wrap=VecAdd
 * so that, without touching their source text:
 *   KO_TIME=<t>      fixes srand(time(NULL)) (kth-problem-seq.c:23,
 *                    TODO-kth-problem-cgm.c:12) -> reproducible runs;
 *   KO_INPUT=<file>  replaces the generated keys, one raw little-endian int32
 *                    per VecAdd call, with the file's keys (kth-problem-seq.c:27,
 *                    TODO-kth-problem-cgm.c:16);
 *   KO_DUMP=<file>   records every key the program appends (to pin the oracle's
 *                    restated generators).
 * ko_env_int() is used only by the parameterised CGM build (n, k from KO_N/KO_K).
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

time_t __real_time(time_t *t);
int __real_VecAdd(void *vector, int element);

time_t __wrap_time(time_t *t)
{
    const char *s = getenv("KO_TIME");
    time_t v = s ? (time_t)strtoll(s, NULL, 10) : __real_time(NULL);
    if (t)
        *t = v;
    return v;
}

static FILE *ko_in, *ko_dump;
static int ko_init;

static void ko_close(void)
{
    if (ko_dump)
        fclose(ko_dump);
    if (ko_in)
        fclose(ko_in);
}

int __wrap_VecAdd(void *vector, int element)
{
    if (!ko_init) {
        ko_init = 1;
        const char *in = getenv("KO_INPUT"), *dump = getenv("KO_DUMP");
        ko_in = in ? fopen(in, "rb") : NULL;
        ko_dump = dump ? fopen(dump, "wb") : NULL;
        atexit(ko_close);
    }
    if (ko_in) {
        int x;
        if (fread(&x, sizeof x, 1, ko_in) == 1)
            element = x;
    }
    if (ko_dump)
        fwrite(&element, sizeof element, 1, ko_dump);
    return __real_VecAdd(vector, element);
}

int ko_env_int(const char *name, int dflt)
{
    const char *s = getenv(name);
    return s ? atoi(s) : dflt;
}
