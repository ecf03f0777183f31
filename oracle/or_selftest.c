/* ORACLE — test infrastructure, NOT product code.
 *
 * Sanitizer driver for the oracle (SURVEY §5 "race / memory checking"): built with
 * -fsanitize=address,undefined by `make -C oracle sanitize` and run by
 * tests/test_oracle_sanitize.py.  It drives every oracle code path the parity tests use:
 *   - FSM-expert episodes (pick_and_place.py:167-277 -> gym step) under all three reward types,
 *     randomized spawns, all 9 tasks, autoreset stream continuation (gym_env.py:477-534);
 *   - all 5 action modes with random in-range actions (gym_env.py:252-281);
 *   - the per-physics-step expert loop (main.py:65-91): plan(1) + actuate + mj_step;
 *   - mj_step from perturbed, interpenetrating states (contact piles, GJK/EPA, overflowing rows).
 * Exit status 0 = clean; the sanitizers abort on the first finding.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define NQ 30
#define NV 27
#define NU 8

static unsigned long long lcg = 0x9e3779b97f4a7c15ULL;
static double urand(void) {
  lcg = lcg * 6364136223846793005ULL + 1442695040888963407ULL;
  return (double)(lcg >> 11) * (1.0 / 9007199254740992.0);
}

static const int TASK_OBJ[9] = {0, 0, 0, 1, 1, 1, 2, 2, 2};
static const int TASK_BIN[9] = {0, 1, 2, 0, 1, 2, 0, 1, 2};

static int expert_episode(or_env* e) {
  int obj, bin, steps = 0;
  or_get_task(e, &obj, &bin);
  or_fsm_init(e, 1, &obj, &bin);
  for (int k = 0; k < 500; k++) {
    if (or_fsm_plan(e, 16) == 10) break; /* S_DONE */
    int st, ti, settle, go;
    double tgt[3];
    or_fsm_get(e, &st, &ti, &settle, tgt, &go);
    float a[10] = {(float)tgt[0], (float)tgt[1], (float)tgt[2], (float)go};
    float obs[85], rc[6];
    int term, trunc, succ;
    or_step(e, a, obs, &term, &trunc, &succ, rc);
    for (int i = 0; i < 85; i++)
      if (!isfinite(obs[i])) { fprintf(stderr, "non-finite obs[%d]\n", i); exit(2); }
    steps++;
    if (term || trunc) break;
  }
  return steps;
}

int main(int argc, char** argv) {
  const int episodes = argc > 1 ? atoi(argv[1]) : 2;
  const double sx[2] = {-0.20, 0.20}, sy[2] = {0.30, 0.45};
  long total = 0;

  /* 1. expert episodes, every reward type, randomized spawns over the 9-task pool */
  for (int rt = 0; rt < 3; rt++) {
    or_env* e = or_create(0, rt, 500, 1, sx, sy, 224);
    or_set_task_pool(e, 9, TASK_OBJ, TASK_BIN);
    float obs[85];
    or_reset(e, 1, 42 + rt, -1, -1, obs);
    for (int ep = 0; ep < episodes; ep++) {
      if (ep) or_reset(e, 0, 0, -1, -1, obs); /* stream continuation */
      total += expert_episode(e);
    }
    or_destroy(e);
  }

  /* 2. every action mode, random actions */
  static const int dims[5] = {4, 8, 10, 8, 10};
  for (int m = 0; m < 5; m++) {
    or_env* e = or_create(m, m % 3, 40, 1, sx, sy, 224);
    float obs[85], rc[6];
    or_reset(e, 1, 7 + m, -1, -1, obs);
    for (int k = 0; k < 12; k++) {
      float a[10] = {0};
      for (int i = 0; i < dims[m]; i++) a[i] = (float)(2.0 * urand() - 1.0);
      if (m == 0) { a[0] *= 0.4f; a[1] = 0.3f + 0.3f * a[1]; a[2] = 0.3f + 0.1f * a[2]; }
      if (m == 1 || m == 2) { a[0] *= 0.3f; a[1] = 0.45f + 0.1f * a[1]; a[2] = 0.4f + 0.1f * a[2]; }
      if (m >= 3) { a[0] *= 0.02f; a[1] *= 0.02f; a[2] *= 0.02f; }
      a[dims[m] - 1] = (float)(urand() > 0.5);
      int term, trunc, succ;
      or_step(e, a, obs, &term, &trunc, &succ, rc);
      total++;
      if (term || trunc) or_reset(e, 0, 0, -1, -1, obs);
    }
    or_destroy(e);
  }

  /* 3. per-physics-step expert (main.py:65-91) */
  {
    or_env* e = or_create(0, 2, 500, 0, sx, sy, 224);
    or_reset_keyframe(e);
    const int o = 0, b = 2;
    or_fsm_init(e, 1, &o, &b);
    for (int k = 0; k < 1500; k++) {
      if (or_fsm_plan(e, 1) == 10) break;
      or_fsm_actuate(e);
      or_mj_step(e);
      total++;
    }
    or_destroy(e);
  }

  /* 4. mj_step from perturbed piles: cubes dropped into each other, on the fingers, into the table */
  {
    or_env* e = or_create(0, 0, 500, 0, sx, sy, 224);
    for (int trial = 0; trial < 6; trial++) {
      or_reset_keyframe(e);
      double qpos[NQ], qvel[NV], ctrl[NU], ws[NV];
      or_get_state(e, qpos, qvel, ctrl, ws);
      for (int c = 0; c < 3; c++) {
        double* p = &qpos[9 + 7 * c];
        p[0] = 0.02 * (urand() - 0.5) + (trial & 1 ? 0.0 : -0.15 + 0.15 * c) * 0.2;
        p[1] = 0.45 + 0.02 * (urand() - 0.5);
        p[2] = 0.235 + 0.035 * c * (trial % 3) / 2.0; /* stacked, slightly interpenetrating */
        double q[4] = {1 + urand(), urand() - 0.5, urand() - 0.5, urand() - 0.5};
        double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int i = 0; i < 4; i++) p[3 + i] = q[i] / n;
      }
      for (int i = 0; i < NV; i++) qvel[i] = 0.2 * (urand() - 0.5);
      or_set_state(e, qpos, qvel, ctrl, ws);
      for (int k = 0; k < 40; k++) {
        or_mj_step(e);
        total++;
      }
      or_get_state(e, qpos, qvel, ctrl, ws);
      for (int i = 0; i < NQ; i++)
        if (!isfinite(qpos[i])) { fprintf(stderr, "non-finite qpos after pile %d\n", trial); return 2; }
    }
    or_destroy(e);
  }
  printf("oracle selftest ok: %ld steps\n", total);
  return 0;
}
