/* TEST INFRASTRUCTURE ONLY (oracle/_ref harness).
 *
 * The reference is built with -finit-real=zero (config.user:25): its never-assigned automatic
 * arrays start at 0.  amdflang has no such flag, and rhs_layer_shear_stress
 * (mod_create_rhs_mlswe.F90:146-279, ad_mlswe > 0) reads one: tau_u(nlayers+1) and
 * tau_v(nlayers+1) are never assigned (:160,246-258).  The harness links with
 * -Wl,--wrap=<that routine>, so momentum_mass's call (mod_splitting.F90:265) enters this
 * wrapper, which zero-fills the stack the routine's frame is about to occupy and then calls the
 * reference routine unchanged (__real_...): the unassigned entries read 0, as in the reference
 * build.  No reference source is copied or modified. */
#include <stddef.h>
#include <string.h>

void __real__QMmod_create_rhs_mlswePrhs_layer_shear_stress(double *rhs_stress, const double *q_df);

static void __attribute__((noinline)) zero_stack_below(size_t n) {
  char buf[n];
  memset(buf, 0, n);
  __asm__ volatile("" : : "r"(buf) : "memory");
}

void __wrap__QMmod_create_rhs_mlswePrhs_layer_shear_stress(double *rhs_stress, const double *q_df) {
  zero_stack_below((size_t)1 << 20);
  __real__QMmod_create_rhs_mlswePrhs_layer_shear_stress(rhs_stress, q_df);
}
