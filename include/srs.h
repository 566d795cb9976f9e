/* Drop-in for the reference's src/srs.h: the KZG structured reference string and the
 * commitment MSM (src/srs.h:11-68).  Same guard, SRS layout and names.  srs_eval_at_s --
 * 9 calls per proof, the prover's dominant cost -- runs on the GPU through plk_msm_g1
 * (include/plonkhip.h), a toy-size call on the host (plk_host.h); the reference's degree check
 * and exit() stay on the host.
 * srs_create reproduces the reference exactly, including that every G1 entry is a
 * multiple of the IDENTITY (src/srs.h:27-36, pinned by src/srs-test.c:15-17). */
#ifndef SRS_H
#define SRS_H

#include <stdio.h>
#include <stdlib.h>

#include "g1.h"
#include "g2.h"
#include "poly.h"
#include "plonkhip.h"

typedef struct {
  G1 *g1s;    /* [1, s, s^2, ..., s^n] * base */
  size_t len; /* n + 1 */
  G2 g2_1;
  G2 g2_s;
} SRS;

static inline SRS srs_create(GF secret, size_t n) {
  SRS srs;
  srs.len = n + 1;
  srs.g1s = (G1 *)malloc(srs.len * sizeof(G1));
  if (!srs.g1s) {
    fprintf(stderr, "Mamory allocation failed in srs_create\n");
    exit(EXIT_FAILURE);
  }
  G1 base = g1_identity();
  GF sp = secret;
  for (size_t i = 0; i < srs.len; i++) {
    srs.g1s[i] = g1_mul(&base, sp.value);
    sp = gf_mul(sp, secret);
  }
  srs.g2_1 = g2_generator();
  srs.g2_s = g2_mul(srs.g2_1, secret.value);
  return srs;
}

static inline void srs_free(SRS *srs) {
  free(srs->g1s);
  srs->g1s = NULL;
  srs->len = 0;
}

/* GPU: sum_i coeffs[i] * g1s[i] (reference: serial g1_mul/g1_add fold); toy sizes: that fold on the host */
static inline G1 srs_eval_at_s(const SRS *srs, const POLY *vs) {
  if (vs->len > srs->len) {
    fprintf(stderr, "Poynomial degree exceeds SRS size: POLY degree: %zu, SRS supports up to degree: %zu \n",
            vs->len, vs->len);
    exit(EXIT_FAILURE);
  }
  if (plk_host_small_(plk_host_mul_(300, vs->len))) return plk_host_msm(srs->g1s, vs->coeffs, vs->len);
  G1 out;
  int rc = plk_msm_g1((const uint8_t *)srs->g1s, (const uint8_t *)vs->coeffs, vs->len, (uint8_t *)&out);
  if (rc != PLK_OK) {
    fprintf(stderr, "srs_eval_at_s failed on the GPU (libplonkhip error %d): %s\n", rc, plk_last_error());
    exit(EXIT_FAILURE);
  }
  return out;
}

#endif /* SRS_H */
