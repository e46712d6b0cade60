/* ctr_oracle.h -- TEST INFRASTRUCTURE ONLY (see ctr_oracle.c header). */
#ifndef CTR_ORACLE_H
#define CTR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One 3-tube system, restated from envs/CTR_Python/Tube.py:7-19 (I, J derived on the host
 * by oracle.py exactly as Tube.__init__ does). Index 0 = innermost tube. */
typedef struct {
    double L[3], Lc[3], E[3], G[3], I[3], J[3], Ux[3], Uy[3];
} oracle_system_t;

void oracle_fk(const float *joints, const int32_t *sys_idx, int64_t n, const oracle_system_t *systems,
               double *tip, int32_t *nfev, int32_t *nstep, int32_t *nseg, int32_t *status);
void oracle_fk_ex(const float *joints, const int32_t *sys_idx, int64_t n, const oracle_system_t *systems,
                  int integrator, int steps_per_m, int rigid,
                  double *tip, int32_t *nfev, int32_t *nstep, int32_t *nseg, int32_t *status);
void oracle_step_ex(int64_t n, const oracle_system_t *systems, const int32_t *sys_idx,
                    float *joints, const float *actions, const double *desired, int32_t *t,
                    const double *tol, int n_substeps, int max_steps, int constrain_alpha,
                    int multi, int egocentric, int integrator, int steps_per_m, int rigid,
                    double *achieved, double *obs, double *reward,
                    uint8_t *done, uint8_t *success, double *error, int32_t *nfev);
void oracle_step(int64_t n, const oracle_system_t *systems, const int32_t *sys_idx,
                 float *joints, const float *actions, const double *desired, int32_t *t,
                 const double *tol, int n_substeps, int max_steps, int constrain_alpha,
                 int multi, int egocentric, double *achieved, double *obs, double *reward,
                 uint8_t *done, uint8_t *success, double *error, int32_t *nfev);
void oracle_set_action(int64_t n, const oracle_system_t *systems, const int32_t *sys_idx,
                       float *joints, const float *actions, int n_substeps, int constrain_alpha);
void oracle_sample_joints(int64_t n, const oracle_system_t *systems, const int32_t *sys_idx,
                          uint64_t seed, const uint32_t *epoch, uint32_t stream, int64_t env_base,
                          float *joints, int32_t *tries);
void oracle_philox(uint32_t *ctr4, uint64_t seed);
void oracle_segments(const float *joints, const int32_t *sys_idx, int64_t n, const oracle_system_t *systems,
                     int32_t *m, double *S);
void oracle_domain_systems(int64_t n, const oracle_system_t *systems, const double *din, const double *dout,
                           const int32_t *sys_idx, double rnd, uint64_t seed, const uint32_t *epoch,
                           int64_t env_base, oracle_system_t *out);
void oracle_jacobian(const double *joints, const int32_t *sys_idx, int64_t n, const oracle_system_t *systems,
                     int integrator, int steps_per_m, int rigid, double eps, double *tip, double *jac);
void oracle_fk_shape(const float *joints, const int32_t *sys_idx, int64_t n, const oracle_system_t *systems,
                     int cap, double *tip, double *r, double *s, int32_t *npts, int32_t *status);
void oracle_fk_segattempts(const float *joints, const int32_t *sys_idx, int64_t n, const oracle_system_t *systems,
                           int32_t *att);
int oracle_version(void);

#ifdef __cplusplus
}
#endif
#endif
