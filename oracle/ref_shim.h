/* ref_shim.h -- forced include for the parameterised reference CGM build only
 * (oracle/build_ref.sh).  TEST INFRASTRUCTURE ONLY. */
int ko_env_int(const char *name, int dflt);
