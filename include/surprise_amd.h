/*
 * surprise_amd.h -- C ABI of the MI355X matrix-factorization SGD library
 * (libsurprise_amd.so, built from surprise_amd/csrc/mf_kernels.hip for gfx950).
 *
 * The reference (nickmvincent/Surprise) has no native ABI: its hot loop is the
 * Cython method SVD.sgd / SVDpp.sgd, reached from Python through AlgoBase.fit().
 * Each entry point below replaces one piece of that loop; the Python host
 * (surprise_amd/matrix_factorization.py) binds them with ctypes exactly where
 * the reference calls self.sgd(trainset) and self.estimate(u, i).
 *
 * Conventions (all entry points):
 *   - every array pointer is a DEVICE pointer (e.g. torch.Tensor.data_ptr());
 *   - no allocation, no host synchronisation, no exceptions cross the ABI;
 *   - calls are ordered on `stream` (a hipStream_t passed as void*; NULL = legacy default);
 *   - return 0 on success, otherwise a hipError_t code or one of MF_E_* below;
 *     mf_last_error() returns a static message for the last failure on this thread;
 *   - factor tables are row-major.  User rows pu[u] and implicit rows yj[j] have leading
 *     dimension ldu >= n_factors; item rows have ldq >= n_factors + 1 and hold the item bias in
 *     column n_factors: qb[i] = [q_i | b_i | 0 ...].  Padding columns must be zero and stay zero;
 *   - item tables (qb, yj) must be < 2 GiB - 4 KiB (32-bit buffer offsets: a masked lane's
 *     offset is the row's offset plus the table size);
 *   - `dtype` selects the arithmetic type of every floating array: MF_F32 or MF_F64.
 */
#ifndef SURPRISE_AMD_H
#define SURPRISE_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MF_F32 0
#define MF_F64 1

/* Item-side update schedule of the epoch kernels. */
#define MF_MODE_PLAIN  0 /* shared item table, plain load/store (lock-free Hogwild!; with one wave
                            the exact sequential order of the reference)                           */
#define MF_MODE_ATOMIC 1 /* shared item table, item deltas applied with float atomics              */
#define MF_MODE_LOG    2 /* item table read-only for the epoch-chunk, every rating's item
                            gradient g = err * pe (pe = the user row [+ u_impl], 1 in the bias
                            column) written to a log (row = CSR position), folded into the table by
                            mf_log_reduce + mf_log_apply: race-free, independent of scheduling     */

#define MF_E_ARG          1001 /* invalid argument (shape, mode, dtype, n_factors too large)      */
#define MF_E_UNSUPPORTED  1002 /* combination not compiled                                       */

#define MF_MAX_FACTORS_F32 512
#define MF_MAX_FACTORS_F64 256

/* Learning rates / regularisation, resolved like SVD.__init__ (matrix_factorization.pyx:140-147)
 * and SVDpp.__init__ (:398-407). global_mean is Trainset.global_mean (trainset.py:252-261),
 * already zeroed by the caller when biased == 0 (matrix_factorization.pyx:238-239). */
typedef struct mf_hyper {
    double lr_bu, lr_bi, lr_pu, lr_qi, lr_yj;
    double reg_bu, reg_bi, reg_pu, reg_qi, reg_yj;
    double global_mean;
} mf_hyper_t;

/* The ratings of one shard, user-major CSR in Trainset.all_ratings() order (trainset.py:180-190):
 * user u's ratings are items[row_ptr[u] .. row_ptr[u+1]) / ratings[...].  `items` and `ratings`
 * are read only inside [row_ptr[0], row_ptr[n_users]). */
typedef struct mf_csr {
    const int64_t *row_ptr;  /* [n_users + 1]                     */
    const int32_t *items;    /* [nnz] item inner ids              */
    const void *ratings;     /* [nnz] dtype, offset applied       */
    int32_t n_users;
    int32_t n_items;
} mf_csr_t;

/*
 * One epoch-chunk of SVD SGD over the users listed in sched[0..n_sched), heaviest first (the
 * waves of users with more than 1/8 of sched[0]'s ratings get raised issue priority).
 * Replaces the body of SVD.sgd's epoch loop (matrix_factorization.pyx:241-262):
 * each wavefront owns a user (pu[u], bu[u] live in registers, updated in the
 * reference's per-rating order); the item rows qb[i] = [q_i | b_i] are updated per `mode`.
 *   pu [n_users][ldu], bu [n_users], qb [n_items][ldq]
 *   biased    : 0 reproduces SVD(biased=False) (hp->global_mean must then be 0)
 *   mode      : MF_MODE_*; MF_MODE_LOG with ldq * sizeof(dtype) <= 1 KiB (the lookahead body)
 *               needs ldq >= n_factors + 2 and qb[i][n_factors + 1] = 1 for every item (the user
 *               bias rides in that column of the user row; the column is never updated)
 *   qlog      : MF_MODE_LOG: device [nnz][ldq] gradient log, row k = err_k * [p_u | 1 | 0..] of
 *               rating k of the CSR (the user row before the rating's step; whole rows written,
 *               zero padding included); each user's segment must be < 2^30
 *               bytes (|I_u| * ldq * sizeof(dtype)).  Other modes: NULL.
 *   elog      : NULL, or (MF_MODE_LOG, ldq * sizeof(dtype) <= 1 KiB) the checkpoint form of the
 *               log: device [nnz + mf_ckpt_interval()] errors, elog[k] = err_k, and qlog holds
 *               one PACKED row per pair of a user's ratings: pair m (ratings row_ptr[u] + 2m,
 *               + 2m + 1) is qlog row (row_ptr[u] + u + 1) / 2 + m and holds [p_u | 1 | 0..]
 *               AFTER the pair's first rating (= before its second; for a user's odd last
 *               rating the final row); qlog then has (row_ptr[n_users] + n_users + 1) / 2 rows
 *               (about half of nnz); mf_log_replay rebuilds the gradients.  Requires
 *               1 - lr_pu * reg_pu != 0 (the replay undoes one step).
 *   n_waves   : wavefronts to launch (<= 0: library default = fill the GPU);
 *               1 with MF_MODE_PLAIN gives the exact sequential reference order when
 *               sched = 0..n_users-1.
 *   flags     : MF_EPOCH_DUP_ITEMS if some user lists the same item twice (in-register
 *               forwarding in MF_MODE_PLAIN / MF_MODE_ATOMIC; MF_MODE_LOG reads the snapshot row);
 */
#define MF_EPOCH_DUP_ITEMS   1
/* flags bits 8..15: XCD mask (bit x: only the launch's wavefronts on XCD x take users, the others
 * exit at once; 0 = every XCD).  Lets two concurrent launches keep to disjoint XCDs, i.e.
 * disjoint L2 caches (the SVD epoch's heaviest users beside the rest). */
#define MF_EPOCH_XCD_SHIFT   8
/* mf_svdpp_epoch, MF_MODE_ATOMIC with ycbuf, rows of <= 1 KiB: one user chain per workgroup
 * (n_waves = chains) whose q deltas go through an LDS ring to three waves that issue the float
 * atomics; sched entries < 0 are skipped (a schedule laid out per chain, strided by n_waves). */
#define MF_EPOCH_SVDPP_HELPERS 2
/* with MF_EPOCH_SVDPP_HELPERS: ONE helper wave per chain (a workgroup of two waves) instead of
 * three -- twice the chains per CU in the same registers (n_waves = chains, as above). */
#define MF_EPOCH_SVDPP_ONE_HELPER 32
/* mf_svd_epoch / mf_svd_epoch_sq with the checkpoint log (elog): err_k is written into its pair's
 * checkpoint row, padding column E + (k - c) (E = n_factors + 2 rounded up to even for fp32,
 * n_factors + 2 for fp64; needs E + 2 <= ldq) instead of elog[k]; mf_log_replay with the same
 * flag reads it there (no per-rating gather of elog). */
#define MF_EPOCH_ERR_IN_ROW 4
/* mf_svd_epoch / mf_svd_epoch_sq with the checkpoint log (elog, errors in elog): the checkpoint
 * rows hold the n_factors factor columns only, at a stride of n_factors (fp32: rounded up to
 * even) elements instead of ldq -- rows of whole cache lines when n_factors * size is a multiple
 * of 128 B (K=128 fp32: 512 B vs 576); the log then needs ck_row0 rows of that stride.
 * mf_log_replay with the same flag reads them so (the bias column's gradient, err_k * 1, is
 * summed from the errors). */
#define MF_EPOCH_CKPT_NARROW 16
/* mf_svd_epoch / mf_svd_epoch_sq (checkpoint log) and mf_svdpp_epoch_qlog: the log rows are
 * stored non-temporal (nt: streamed past L2 / MALL), so a log far larger than the MALL does not
 * evict the item rows the epoch gathers (C4: the epoch kernel 18.0 -> 14.6 ms). */
#define MF_EPOCH_LOG_NT 64
/* mf_log_replay flags bits 16..23: the launch's waves per CU (0: the default, 16) */
#define MF_REPLAY_WPC_SHIFT 16
int mf_svd_epoch(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                 int32_t ldu, void *qb, int32_t ldq, int32_t n_factors, int32_t biased,
                 const mf_hyper_t *hp, int32_t mode, void *qlog, void *elog, int32_t n_waves,
                 int32_t flags, int32_t dtype, void *stream);

/*
 * One epoch-chunk of SVD++ SGD (SVDpp.sgd epoch body, matrix_factorization.pyx:463-498) in the
 * exact per-user affine form: per user, one gather of y_j (j in I_u), the sequential rating
 * loop with u_impl maintained incrementally, and one affine write-back y_j <- A y_j + c
 * (stores in MF_MODE_PLAIN, float atomics of (A-1) y_j + c otherwise).  yj [n_items][ldu].
 * Always biased (SVDpp has no option).  status (nullable device int32, MF_EPOCH_SVDPP_HELPERS
 * only; zeroed by the caller, OR-ed by the kernel): bit MF_HX_HELPER_TIMEOUT -- a helper wave
 * waited past its bound and stopped, q deltas were lost, the item table is invalid;
 * bit MF_HX_CHAIN_FALLBACK -- a chain found no room in its ring within the bound and issued a
 * bank's atomics itself (results intact).  Every wait is bounded: nothing hangs the GPU.
 */
#define MF_HX_HELPER_TIMEOUT 1
#define MF_HX_CHAIN_FALLBACK 2
/* hot (nullable, MF_EPOCH_SVDPP_HELPERS only): per item, nonzero = the row has a delta replica at
 * row n_items + i of qb (qb then holds 2 * n_items rows, the replica rows zero at the call and
 * 3 * n_items * ldq * size < 2^32).  The float atomics on one row are performed one after the
 * other at the memory side, so the most-rated items' rows bound the launch; the chains of odd
 * workgroups add a hot item's deltas to its replica, the others to the row, and every read of a
 * hot row adds the replica -- the value one row would hold.  mf_svdpp_hot_fold afterwards. */
int mf_svdpp_epoch(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu, void *bu,
                   int32_t ldu, void *qb, int32_t ldq, void *yj, int32_t n_factors,
                   const mf_hyper_t *hp, int32_t mode, void *qlog, void *ycbuf, int32_t n_waves,
                   int32_t flags, int32_t *status, const uint8_t *hot, int32_t dtype,
                   void *stream);

/*
 * One epoch-chunk of SVD++ SGD (matrix_factorization.pyx:463-498) with the item rows READ-ONLY
 * for the chunk (the q log): the per-user affine form of mf_svdpp_epoch with y deferred (ycbuf,
 * as MF_MODE_ATOMIC with ycbuf: mf_svdpp_y_fold afterwards), and instead of float atomics on
 * q_i / b_i each rating's gradient err_k [p_k + m_k | 1] (m_k: u_impl before rating k; the bias
 * column K holds err_k) is stored as row log_row0[u] + j of qlog ([rows][ldq], j = the rating's
 * index in the user's CSR row; log_row0: int64 per user, valid for the scheduled users).  Fold
 * with mf_log_reduce (perm = the chunk's log rows grouped by item, recency weights) and
 * mf_log_apply, as the SVD gradient log: q_i += lr (S_i - W reg q_i), i.e. the reference's
 * steps on the row to first order (oracle_svdpp_sgd_stalelog, every item stale).  Rows of
 * <= 1 KiB, no repeated items; flags: MF_EPOCH_DUP_ITEMS must be clear, XCD mask bits allowed.
 * n_waves <= 0: one wave per user up to the launch's cap.  A user's log segment must stay below
 * 1 GiB.  user_sq (nullable, fp64 [n_users]): each trained user's |p_u|^2 over the factor
 * columns is stored there (as mf_svd_epoch_sq), so the next chunk's <p^2> is
 * mf_user_sq_reduce's sum instead of an mf_sumsq pass over every user row.
 * Replaces matrix_factorization.pyx:487 / :494-495 (the item-side updates).
 */
int mf_svdpp_epoch_qlog(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu,
                        void *bu, int32_t ldu, void *qb, int32_t ldq, void *yj, int32_t n_factors,
                        const mf_hyper_t *hp, void *qlog, const int64_t *log_row0, void *ycbuf,
                        double *user_sq, int32_t n_waves, int32_t flags, int32_t dtype,
                        void *stream);

/* The hybrid helper-wave launch (MF_EPOCH_SVDPP_HELPERS, three helpers): mf_svdpp_epoch in
 * MF_MODE_ATOMIC, except that the chunk's ratings with cold_row[p] >= 0 (CSR positions p of
 * csr) belong to "cold" items whose rows stay read-only for the chunk: their q / b gradient
 * err_k [s_k | 1] is stored to row cold_row[p] of cold_log ([rows][ldq], rows < 2^31 / (ldq *
 * size)), and only the other items' deltas go to the helper waves' float atomics.  The caller
 * folds the cold log after the chunk (mf_log_reduce over the cold items' row ranges with their
 * recency weights, mf_log_apply with the cold items' counts: oracle_svdpp_sgd_stalelog with the
 * cold items stale).  user_sq[u] = |p_u|^2 of every trained user (the fold's <p^2>). */
int mf_svdpp_epoch_mix(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu,
                       void *bu, int32_t ldu, void *qb, int32_t ldq, void *yj, int32_t n_factors,
                       const mf_hyper_t *hp, void *cold_log, const int32_t *cold_row,
                       void *ycbuf, double *user_sq, int32_t n_waves, int32_t flags,
                       int32_t *status, const uint8_t *hot, int32_t dtype, void *stream);

/* After mf_svdpp_epoch with hot rows: row i += row n_items + i and the replica row zeroed, for
 * i in hot_items[0 .. n_hot). */
int mf_svdpp_hot_fold(void *qb, int32_t ldq, int32_t n_items, const int32_t *hot_items,
                      int32_t n_hot, int32_t dtype, void *stream);

/*
 * SVD++ deferred y update (MF_MODE_ATOMIC with ycbuf != NULL in mf_svdpp_epoch): the epoch kernel
 * stores every user's affine-update vector c_u in ycbuf [n_users][ldu] instead of applying
 * y_j <- A_u y_j + c_u.  This composes, per item j, the maps of the users item_users[x] for x in
 * the item's pieces (piece p = [piece_beg[p], piece_beg[p+1]), <= 64 entries; the item's pieces
 * [item_piece_ptr[j], item_piece_ptr[j+1]); users in CSR order), applying them to y_j one user
 * after the other.  uA [n_users] = A_u = (1 - lr_yj reg_yj)^{|I_u|}; piece_c [n_pieces][ldu] and
 * piece_A [n_pieces] are scratch.  Race-free and deterministic (a fixed two-level tree).
 * piece_item (nullable, [n_pieces]: each piece's item): an item with ONE piece gets its map
 * applied by the piece's own wave (no scratch round trip, the same arithmetic), the per-item pass
 * then composes only the items of several pieces.
 */
int mf_svdpp_y_fold(void *yj, int32_t ldu, int32_t n_factors, const void *ycbuf, const void *uA,
                    const int32_t *item_users, const int32_t *piece_beg, int64_t n_pieces,
                    const int32_t *item_piece_ptr, int32_t n_items, void *piece_c,
                    void *piece_A, const int32_t *piece_item, int32_t dtype, void *stream);

/* stat[0] += sum of x[r][c]^2 over r < n_rows, c < n_cols, stat[1] += n_rows * n_cols (x is
 * [n_rows][ld]; stat is two device doubles; both parts add up across ranks).  <pu^2> =
 * stat[0] / stat[1] is the statistic of the count-aware merge rules. */
int mf_sumsq(const void *x, int64_t n_rows, int32_t n_cols, int32_t ld, double *stat,
             int32_t dtype, void *stream);

/*
 * Recency weights of a chunk's logged gradients (mf_log_reduce / mf_log_replay, then
 * mf_log_apply with MF_MERGE_RECENCY): the gradient of a rating at position pos among the
 * chunk's N ratings of its item (users in order, every rank) is weighted by (1 - eta)^(N-1-pos),
 * eta = lr_qi (<p^2> + reg_qi) in factor columns and lr_bi (1 + reg_bi) in the bias column
 * (n_factors), <p^2> = p2stat[0] / p2stat[1] -- the sequential reference's steps on the row, to
 * first order.
 */
typedef struct mf_recency {
    const int32_t *rpos;    /* [perm entries] the rating's position among this rank's ratings of
                               its item in the chunk (users in order)                         */
    const int32_t *pos0;    /* [n_items], nullable: the chunk's ratings of the item on earlier
                               ranks (added to rpos)                                          */
    const int32_t *totals;  /* [n_items] N: the chunk's ratings of the item on every rank      */
    const double *p2stat;   /* {sum p^2, count} at the chunk start, every rank                */
} mf_recency_t;

/*
 * Delta-log merge, step 1 (MF_MODE_LOG): sums[p][c] = sum_{x in [piece_beg[p], piece_beg[p+1])}
 * w_x qlog[perm[x]][c] for c < n_cols (zero for n_cols <= c < ld), summed in x order.  perm lists
 * the chunk's log rows grouped by item; an item's rows are cut into consecutive pieces of 1..64
 * rows.  rec NULL: w = 1; else the recency weights (piece_item and hp required; the bias column
 * is n_cols - 1).
 */
int mf_log_reduce(const void *qlog, int32_t ld, int32_t n_cols, const int32_t *perm,
                  const int32_t *piece_beg, int64_t n_pieces, void *sums,
                  const int32_t *piece_item, const mf_hyper_t *hp, const mf_recency_t *rec,
                  int32_t dtype, void *stream);

/*
 * Delta-log merge, step 1 for the checkpoint form (mf_svd_epoch with elog): the same sums as
 * mf_log_reduce would give on the gradient log, sums[p][c] = sum over the piece's ratings k of
 * err_k * p_k[c] (c <= n_factors; 0 above), where p_k comes from its pair's packed checkpoint
 * row: ck_pos[x] = 2 * row + (k - row_ptr[u]) mod 2 (x = the rating's index in perm; row as in
 * mf_svd_epoch's elog), which holds the user row after the pair's first rating c: for k = c + 1
 * (odd) the row itself, for k = c the epoch kernel's step undone,
 * p_k = (row - err_k * lr_pu * q_{item(k)}) / ap (ap = 1 - lr_pu * reg_pu on factor columns;
 * q from the snapshot table qb; every rating of a piece has the same item) -- call it before
 * mf_log_apply.  piece_item (nullable): the item of each piece (else read through perm and the
 * CSR items).  Requires ldq * sizeof(dtype) <= 1 KiB (narrow rows: their n_factors columns
 * <= 1 KiB, ldq <= 1.5 KiB -- fp64 K = 128).  flags: bits 8..15 an XCD mask as in
 * mf_svd_epoch (MF_EPOCH_XCD_SHIFT), 0 = every XCD; bits 16..23 the launch's waves per CU
 * (MF_REPLAY_WPC_SHIFT; 0 = 16); MF_EPOCH_ERR_IN_ROW: errors in the rows;
 * MF_EPOCH_CKPT_NARROW: narrow checkpoint rows.  Unlike mf_log_reduce, a piece may hold any
 * number >= 1 of ratings (of one item): longer pieces mean fewer sums rows for mf_log_apply.
 * rec (nullable): each gradient err_k * p_k weighted by its recency weight (mf_recency_t).
 */
int mf_log_replay(const void *qlog, const void *elog, int32_t ldq, int32_t n_factors,
                  const mf_csr_t *csr, const void *qb, const mf_hyper_t *hp, const int32_t *perm,
                  const int32_t *ck_pos, const int32_t *piece_beg, int64_t n_pieces, void *sums,
                  const int32_t *piece_item, const mf_recency_t *rec, int32_t flags,
                  int32_t dtype, void *stream);

/*
 * mf_svd_epoch in MF_MODE_LOG with the checkpoint log (elog != NULL, the lookahead body), also
 * keeping user_sq current: user_sq[u] = sum_{c < n_factors} p_u[c]^2 (fp64) of every trained
 * user's row after the epoch -- the <p^2> statistic of the log fold's count-aware weights
 * without another pass over pu (mf_user_sq_reduce).  Same item-side results as mf_svd_epoch.
 * item_bias (nullable, [n_items] of dtype): with MF_EPOCH_CKPT_NARROW rows whose factor columns
 * fill whole 512-B lane groups (fp32 K=128, fp64 K=64 / 128), the item biases are read from
 * item_bias[i] -- a mirror of qb[i][n_factors], kept by mf_log_apply's bias_out -- instead of
 * from the row, so a row gather touches only its factor lines (with ldq a multiple of 128 B).
 */
int mf_svd_epoch_sq(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu,
                    void *bu, int32_t ldu, void *qb, int32_t ldq, int32_t n_factors, int32_t biased,
                    const mf_hyper_t *hp, void *qlog, void *elog, double *user_sq,
                    const void *item_bias, int32_t n_waves, int32_t flags, int32_t dtype,
                    void *stream);

/*
 * mf_svd_epoch_sq for the heaviest users by a blocked solve (replaces the same loop,
 * matrix_factorization.pyx:241-262, for the users it is given): one workgroup per user; over
 * every block of 16 ratings the errors are the solution of a unit lower-triangular system built
 * from the block's item-row Gram matrix (MFMA) and the row at the block's start, so the
 * sequential chain per rating is one readlane + FMA instead of two 64-lane reductions.  Writes
 * exactly what mf_svd_epoch_sq with MF_EPOCH_ERR_IN_ROW writes for those users (the user's row
 * and bias, its packed checkpoint rows with their errors, user_sq[u]) -- equal up to rounding.
 * Needs the MF_MODE_LOG item layout (column n_factors + 1 of qb = 1), ldq >= n_factors + 4
 * (fp32: the error columns, as MF_EPOCH_ERR_IN_ROW), ldq * size <= 1 KiB, no user listing an
 * item twice.  n_blocks: workgroups of the launch (0: one per scheduled user; users are taken
 * strided); flags: MF_EPOCH_XCD_SHIFT's mask only.
 */
int mf_svd_epoch_gram(const mf_csr_t *csr, const int32_t *sched, int64_t n_sched, void *pu,
                      void *bu, int32_t ldu, const void *qb, int32_t ldq, int32_t n_factors,
                      int32_t biased, const mf_hyper_t *hp, void *qlog, double *user_sq,
                      int32_t n_blocks, int32_t flags, int32_t dtype, void *stream);

/* user_sq[r] = sum_{c < n_cols} x[r * ld + c]^2 (fp64) for r < n_rows: initial user_sq. */
int mf_user_sq(const void *pu, int64_t n_rows, int32_t n_cols, int32_t ld, double *user_sq,
               int32_t dtype, void *stream);

/* The {sum, count} statistic buffers below (out, stat_next) hold 2 doubles, plus MF_SQ_PARTS
 * doubles of scratch after them when n_rows / n_users >= MF_SQ_PARTS_MIN: above that size the
 * sum runs as MF_SQ_PARTS fixed-range partial sums (a launch of its own, on the same stream)
 * added in order -- still bit-reproducible, at the chip's bandwidth instead of one workgroup's. */
#define MF_SQ_PARTS 256
#define MF_SQ_PARTS_MIN 65536

/* out[0] = sum of user_sq[0..n_rows) in a fixed order, out[1] = n_rows * n_cols: the {sum,
 * count} pair mf_sumsq accumulates (here written, not added; bit-reproducible).  out: 2 doubles
 * (+ MF_SQ_PARTS scratch from MF_SQ_PARTS_MIN rows). */
int mf_user_sq_reduce(const double *user_sq, int64_t n_rows, int32_t n_cols, double *out,
                      void *stream);

/* Checkpoint interval of the checkpoint log (ratings per stored user row). */
int mf_ckpt_interval(void);

/* The item layout of one SVD++ q-log epoch-chunk for mf_svdpp_qlog_fold, in item-grouped
 * positions (the chunk's ratings grouped by item, users in order within an item).  Cold items
 * (at most a few rows: one wavefront takes them in turn) list their rows directly; hot items
 * (more rows) are cut into pieces of <= 64 rows, summed / composed per piece by the launch's two
 * pre-passes first.  An item is either cold or hot. */
typedef struct mf_qlog_fold {
    const int32_t *perm;          /* cold items' log rows, by item                               */
    const int32_t *rpos;          /* [perm entries] the row's position among its item's rows     */
    const int32_t *item_row_beg;  /* [n_items + 1] item i's cold rows: perm[beg[i] .. beg[i+1]),
                                     at most 64 of them                                         */
    const int32_t *users;         /* [perm entries] each cold row's rater (CSR order)           */
    const int32_t *hot_perm, *hot_rpos, *hot_users;  /* hot items' rows / positions / raters     */
    const int32_t *hot_piece_beg;       /* [n_hot_pieces + 1] pieces of <= 64 hot positions     */
    const int32_t *hot_piece_item;      /* [n_hot_pieces] each piece's item                     */
    const int32_t *hot_item_piece_ptr;  /* [n_items + 1] item i's pieces                        */
    int64_t n_hot_pieces;
    void *hot_sums;                     /* scratch [n_hot_pieces][ldq]                          */
    void *hot_piece_c, *hot_piece_A;    /* scratch [n_hot_pieces][ldu], [n_hot_pieces]          */
} mf_qlog_fold_t;

/* One rank's fold of an SVD++ q-log epoch-chunk in ONE pass over the items (replaces
 * mf_log_reduce + mf_log_apply + mf_svdpp_y_fold for mf_svdpp_epoch_qlog's chunks; SVDpp.sgd's
 * item and implicit-factor steps, matrix_factorization.pyx:486-498, in the q log's schedule).
 * Per item i touched by the chunk, one wavefront:
 *   S_i = sum over the item's logged rows x of (1 - eta)^(N_i - 1 - rpos[x]) qlog[perm[x]]
 *         (eta of the bias column in column n_factors; hot items: their pieces' sums),
 *   qb[i] += lr o (S_i - W reg o qb[i])      (MF_MERGE_RECENCY of mf_log_apply; N_i = totals[i]),
 *   yj[i] <- A_u yj[i] + ycbuf[u] for the item's raters u in CSR order (A_u = uA[u]).
 * p2stat: the chunk-start {sum p^2, count} (one rank).  stat_next / user_sq / n_users: as
 * mf_log_apply's.  Rows: qb, qlog [.][ldq], yj, ycbuf [.][ldu]. */
int mf_svdpp_qlog_fold(void *qb, int32_t ldq, int32_t n_factors, void *yj, int32_t ldu,
                       const void *qlog, const mf_qlog_fold_t *lay, const int32_t *totals,
                       const double *p2stat, const mf_hyper_t *hp, const void *ycbuf,
                       const void *uA, int32_t n_items, double *stat_next,
                       const double *user_sq, int64_t n_users, int32_t dtype, void *stream);

/*
 * Delta-log merge, step 2: S_i = sum of sums[p] over p in [item_piece_ptr[i], item_piece_ptr[i+1])
 * (item_piece_ptr NULL: S_i = sums[i], e.g. after an all-reduce), plus -- when sums2 is not NULL
 * (a chunk whose users were logged as two groups, e.g. on two streams) -- the sum of sums2[p] over
 * p in [item_piece_ptr2[i], item_piece_ptr2[i+1]), added in that order.  delta_out (nullable,
 * [n_items][ld]) receives S; apply != 0 turns the summed gradients into the summed item steps,
 * D_i = lr o (S_i - N reg o qb[i])  (lr, reg = lr_qi, reg_qi in columns < n_factors and lr_bi,
 * reg_bi in bias_col; bias_col < 0: none), N = totals[i] (ratings of item i in the chunk, all
 * ranks; required with apply), and adds w * D_i to qb[i]:
 *   MF_MERGE_SUM:   w = 1;
 *   MF_MERGE_COUNT: w = (1 - (1-eta)^N) / (N eta), N = totals[i] (ratings of item i in the chunk,
 *                   all ranks), eta = lr_bi (1 + reg_bi) in bias_col and lr_qi (<p^2> + reg_qi)
 *                   in factor columns, <p^2> = p2stat[0] / p2stat[1] (mf_sumsq's two doubles);
 *   MF_MERGE_RECENCY: the sums carry the recency weights (mf_recency_t); adds
 *                   lr o (S_i - W reg o qb[i]) with W = (1 - (1-eta)^N) / eta, the weights' sum.
 * stat_next (nullable, 2 device doubles -- + MF_SQ_PARTS scratch from MF_SQ_PARTS_MIN users --,
 * not p2stat): user_sq NULL: set to {0, 0} -- the next
 * chunk's mf_sumsq accumulator, cleared here instead of by a separate fill; user_sq != NULL
 * (mf_svd_epoch_sq's array, n_users rows): set to mf_user_sq_reduce's {sum, n_users * n_factors}
 * -- the next chunk's <p^2>, summed inside this launch (every epoch kernel of the chunk must have
 * finished before it).  bias_out (nullable, [n_items], needs apply and bias_col >= 0): also
 * receives each item's new qb[i][bias_col] (mf_svd_epoch_sq's item_bias mirror).
 */
int mf_log_apply(void *qb, int32_t n_items, int32_t ld, int32_t n_factors, int32_t bias_col,
                 const void *sums, const int32_t *item_piece_ptr, const void *sums2,
                 const int32_t *item_piece_ptr2, const int32_t *totals, const mf_hyper_t *hp,
                 const double *p2stat, int32_t rule, void *delta_out, int32_t apply,
                 double *stat_next, const double *user_sq, int64_t n_users, void *bias_out,
                 int32_t dtype, void *stream);

/* Merge rules of mf_item_merge. */
#define MF_MERGE_SUM   0 /* delta = sum_r d_r                                                      */
#define MF_MERGE_COUNT 1 /* count-aware: SUM while a row's steps are small, count-weighted MEAN
                            once they saturate (item factors and biases)                           */
#define MF_MERGE_MEAN  2 /* count-weighted MEAN: sum_r (n_r / N) d_r (SVD++ implicit factors)      */
#define MF_MERGE_RECENCY 3 /* mf_log_apply: sums weighted by recency (mf_recency_t), the default;
                              mf_item_merge: each rank's delta decayed by the later ranks' steps */

/*
 * Item-side merge of an epoch-chunk across ranks for MF_MODE_PLAIN /
 * MF_MODE_ATOMIC tables and SVD++'s yj: `tab` ([n_replicas][n_items][ld]; one copy per rank in
 * the library's own engine) against the chunk-start snapshot `snap` [n_items][ld]:
 *     delta[i] = sum_r w_r(i) (tab_r[i] - snap[i])
 * counts ([n_replicas][n_items]: ratings of item i trained in replica r this chunk) and totals
 * ([n_items]: the same summed over every replica of every rank) give n_r and N.
 *   MF_MERGE_SUM:   w = 1 (counts may be NULL);
 *   MF_MERGE_COUNT: w_r(i) = (n_r/N)(1-(1-eta)^N)/(1-(1-eta)^{n_r}) with eta = lr_bi (1 + reg_bi)
 *                   in column bias_col (-1: none) and eta = lr_qi (<pu^2> + reg_qi) in columns
 *                   < n_factors, <pu^2> being the mean squared entry of pu[:, :n_factors]
 *                   ([n_users][ldu], reduced on the device into `work`, 2 doubles of scratch);
 *   MF_MERGE_MEAN:  w_r(i) = n_r / N;
 *   MF_MERGE_RECENCY (n_replicas 1; counts[i] = N_>r(i), the ratings of item i on the ranks after
 *                   this one in the chunk, totals unused): w(i) = (1-eta)^{N_>r(i)}, eta as for
 *                   MF_MERGE_COUNT -- the ranks' steps composed in rank order, each step decaying
 *                   the row by (1 - eta) to first order, so rank r's delta is carried through the
 *                   later ranks' steps (the reference applies them after it; SVD++'s multi-rank q
 *                   / b merge, oracle_svdpp_sgd_groups_merge(merge=3)).
 * apply != 0: snap += delta and every replica := snap.  apply == 0: only delta_out is written
 * (the caller all-reduces it with RCCL SUM, then calls mf_item_apply).
 */
int mf_item_merge(void *tab, void *snap, int32_t n_items, int32_t ld, int32_t n_factors,
                  int32_t bias_col, int32_t n_replicas, int32_t rule, const int32_t *counts,
                  const int32_t *totals, const mf_hyper_t *hp, const void *pu, int32_t n_users,
                  int32_t ldu, void *work, void *delta_out, int32_t apply, int32_t dtype,
                  void *stream);

/* snap += delta; every replica := snap (second half of a multi-rank merge). */
int mf_item_apply(void *tab, void *snap, int32_t n_items, int32_t ld, int32_t n_replicas,
                  const void *delta, int32_t dtype, void *stream);

/*
 * SVD++ implicit factors across ranks (surprise_amd/dist.py; replaces nothing in the reference,
 * which is single-process).  Rank r's chunk left y_r = A_r y_s + c_r in `tab` (its users' end-of-
 * user maps y_j <- A_u y_j + c_u composed in CSR order, A_u = (1 - lr_yj reg_yj)^{|I_u|}) over the
 * chunk-start snapshot y_s in `snap`.  Ranks own consecutive user ranges, so the single-GPU
 * composition over all users is y = A y_s + sum_r S_r c_r with A = prod_r A_r and
 * S_r = prod_{s>r} A_s (per item).
 *   phase 0: delta = s[i] * (tab - a[i] * snap)   (a = A_r, s = S_r; SUM-all-reduce it after)
 *   phase 1: tab = snap = a[i] * snap + delta      (a = A; s unused)
 * tab, snap, delta [n_items][ld]; a, s [n_items] (dtype).
 */
int mf_item_affine(void *tab, void *snap, int32_t n_items, int32_t ld, const void *a,
                   const void *s, void *delta, int32_t phase, int32_t dtype, void *stream);

/*
 * One epoch of NMF.sgd (matrix_factorization.pyx:646-735) in two race-free passes.
 * mf_nmf_user_pass: one wave per user computes every rating's estimate
 *   est = mu + b_u + b_i + <q_i, p_u>  (biased; the b_u recursion of :707-708 in the user's
 *   order, b_i read from qb's column n_factors as the epoch-start snapshot) or <q_i, p_u>,
 *   saves it in est[k] (k = CSR position) and, biased, the item-bias step in blog[k]; sums the
 *   user's numerator / denominator (:712-713) and writes p_u's multiplicative step (:719-723) to
 *   pu_next (pu itself stays the epoch's factors).  hp: reg_pu, lr_bu, reg_bu, lr_bi, reg_bi,
 *   global_mean (0 when unbiased).
 * mf_nmf_item_pass: one wave per item walks its ratings (csc_ptr[n_items+1], csc_pos[nnz] = CSR
 *   positions in ir order, row_user[nnz] = user of each CSR position), sums p_u r and p_u est over
 *   the OLD pu (:714-716) and takes q_i's step (:726-730) with hp->reg_qi; biased:
 *   b_i += w * sum of blog (rule MF_MERGE_COUNT: w = (1 - (1-eta)^N) / (N eta),
 *   eta = lr_bi (1 + reg_bi); MF_MERGE_SUM: w = 1).  Call it after the user pass, then swap
 *   pu / pu_next.  pu, pu_next [n_users][ldu]; qb [n_items][ldq] = [q_i | b_i | 0 ...].
 *   Optional piece form (rows of <= 64 fp32 / 32 fp64 elements; else ignored): every item's CSC
 *   range cut into pieces of <= 64 ratings, piece p = [piece_beg[p], piece_beg[p+1]) (absolute
 *   CSC positions, n_pieces+1 entries), the item's pieces [item_piece_ptr[i], item_piece_ptr[i+1]);
 *   scratch [n_pieces][2 ldq + 1].  The pieces are reduced in parallel and added per item in
 *   order (deterministic).  piece_beg = NULL: one wave per item.  Optional csc_ratings[nnz] /
 *   csc_user[nnz] (piece form only; NULL: gathered): ratings[csc_pos[x]] and row_user[csc_pos[x]]
 *   stored in CSC order, read coalesced.
 *   mf_nmf_user_pass takes the same piece form when unbiased (the biased b_u recursion is a
 *   chain): the user's CSR range in pieces of <= 64 ratings (absolute CSR positions), the
 *   user's pieces [user_piece_ptr[u], user_piece_ptr[u+1]), piece_user[p] = its user,
 *   scratch [n_pieces][2 ldu].  piece_beg = NULL: one wave per user.
 */
int mf_nmf_user_pass(const mf_csr_t *csr, const void *pu, void *pu_next, void *bu, int32_t ldu,
                     const void *qb, int32_t ldq, int32_t n_factors, int32_t biased,
                     const mf_hyper_t *hp, void *est, void *blog, const int64_t *piece_beg,
                     int64_t n_pieces, const int32_t *user_piece_ptr, const int32_t *piece_user,
                     void *scratch, int32_t dtype, void *stream);
int mf_nmf_item_pass(const int64_t *csc_ptr, const int64_t *csc_pos, const int32_t *row_user,
                     const void *ratings, const void *est, const void *blog, const void *pu,
                     int32_t ldu, void *qb, int32_t ldq, int32_t n_items, int32_t n_factors,
                     int32_t biased, const mf_hyper_t *hp, int32_t rule,
                     const int64_t *piece_beg, int64_t n_pieces, const int32_t *item_piece_ptr,
                     void *scratch, const void *csc_ratings, const int32_t *csc_user,
                     int32_t dtype, void *stream);

/*
 * One epoch of baseline_als (optimize_baselines.pyx:14-54): b_i = sum over ir[i] of
 * (r - mu - b_u) / (reg_i + |ir[i]|) for every item, then b_u = sum over ur[u] of
 * (r - mu - b_i) / (reg_u + |ur[u]|) for every user.  csc as for mf_nmf_item_pass, and the optional
 * CSC-ordered csc_ratings / csc_user the same way (NULL: gathered through csc_pos).
 * (baseline_sgd, :57-84, is mf_svd_epoch with n_factors = 0.)
 */
int mf_baseline_als_epoch(const mf_csr_t *csr, const int64_t *csc_ptr, const int64_t *csc_pos,
                          const int32_t *row_user, void *bu, void *bi, double global_mean,
                          double reg_u, double reg_i, const void *csc_ratings,
                          const int32_t *csc_user, int32_t dtype, void *stream);

/*
 * Batched SVD.estimate (matrix_factorization.pyx:269-299): for x < n, with u[x] < 0 / i[x] < 0
 * meaning an unknown user / item ('UKN__' ids, algo_base.py:137-144):
 *   biased:   est = mu (+bu[u] if known u) (+b_i if known i) (+ q_i.(pu[u] + imp[u]) if both)
 *   unbiased: est = q_i.pu[u] if both known, else impossible[x] = 1 (PredictionImpossible)
 * imp (nullable, [n_users][ldu]) is the SVD++ implicit term per user (mf_svdpp_user_implicit);
 * with it this is SVDpp.estimate (:506-522).  est is dtype, impossible is int32.
 */
int mf_predict(int64_t n, const int32_t *u, const int32_t *i, const void *pu, const void *bu,
               int32_t ldu, const void *qb, int32_t ldq, const void *imp, int32_t n_factors,
               int32_t biased, double global_mean, void *est, int32_t *impossible, int32_t dtype,
               void *stream);

/*
 * accuracy.rmse / accuracy.mae over a batch of estimates (accuracy.py:22-90), finishing each
 * estimate as AlgoBase.predict does (algo_base.py:148-169): impossible[x] (nullable) -> fallback
 * (default_prediction(), the trainset mean), minus `offset`, clipped to [lo, hi]; the true rating
 * is r[x] - offset.  Accumulates out[0] += sum err^2, out[1] += sum |err|, out[2] += n (three
 * device doubles, zeroed by the caller): rmse = sqrt(out[0]/out[2]), mae = out[1]/out[2].
 * est is dtype, r is always fp64 (the reference's r_ui - est is fp64).  Replaces the
 * per-Prediction Python loop of the reference's test() + rmse() (algo_base.py:191-218).
 */
int mf_rating_errors(int64_t n, const void *est, const int32_t *impossible, const void *r,
                     double fallback, double offset, double lo, double hi, double *out,
                     int32_t dtype, void *stream);

/* imp[u] = (sum_{j in I_u} yj[j]) / sqrt(|I_u|)  (SVDpp.estimate :518-520), zero for empty users;
 * yj is replica 0, imp is [n_users][ldu]. */
int mf_svdpp_user_implicit(const mf_csr_t *csr, const void *yj, int32_t ldu, void *imp,
                           int32_t n_factors, int32_t dtype, void *stream);

/* *ok = 1 if the current device deals workgroups round-robin over 8 XCDs (workgroup b on XCD
 * b mod 8, read from the XCC_ID register; checked once per device): the layout the XCD masks
 * of mf_svd_epoch / mf_log_replay (flags bits 8..15) assume.  Masked launches are refused
 * (MF_E_UNSUPPORTED) where it does not hold. */
int mf_xcd_layout(int32_t *ok);

/* The dispatch check of the XCD-masked launches: every masked launch settles each
 * wave's (workgroup's) slot against its grid index in a device-side 64-bit sum that stays 0
 * exactly when the launch's slots were a permutation -- every user / piece processed once.
 * *sum = that sum over every code object of the library (synchronous; read after the device's
 * work).  Nonzero: some masked launch since the library was loaded trained a user twice or
 * never (the engine raises). */
int mf_dispatch_check(uint64_t *sum);

/* Self-test of the XCD id register: out[b] = HW_REG_XCC_ID of workgroup b, b < n_blocks. */
int mf_selftest_xcc(int32_t *out, int32_t n_blocks, void *stream);

/* Self-test of the wavefront reduction: out[w] = sum of in[64w .. 64w+63], w < n_waves. */
int mf_selftest_wave_sum(const void *in, void *out, int32_t n_waves, int32_t dtype, void *stream);

/* Library version (major*10000 + minor*100 + patch) and last error message. */
int mf_version(void);
const char *mf_last_error(void);

/* sha256 (hex) of the sources and compile lines this library was built from
 * (surprise_amd/build.py source_hash()): the Python loader refuses a library whose hash differs
 * from the sources next to it. */
const char *mf_source_hash(void);

/* ---- stream ordering without marker packets (the two-stream SVD step)
 * A HIP event recorded on a stream is a marker packet in its queue; the kernel queued after it
 * starts ~7 us late.  mf_launch_event(ev) binds ev to the NEXT mf_log_apply / mf_log_replay
 * launch of the calling thread as that dispatch's stop event (hipExtLaunchKernel): ev completes
 * with the kernel and the queue holds no marker.  The others are thin wrappers so that a
 * binding needs no HIP headers: create / destroy / record an event (timing disabled), and make
 * a stream wait for one.  Replace the torch.cuda.Event record / wait_event pairs of the
 * engine's fork / join (no reference counterpart: the reference is single-threaded). */
int mf_event_create(void **event);
int mf_event_destroy(void *event);
int mf_event_record(void *event, void *stream);
int mf_stream_wait_event(void *stream, void *event);
int mf_launch_event(void *event);

/* mf_launch_join(words, role, epoch): the next mf_log_replay launch of the calling thread takes
 * part in an in-kernel join (no barrier packet in the main stream's queue): role 1 (the light
 * replay on the side stream) publishes `epoch` into words[576] when its last block has stored its
 * sums; role 2 (the heavy replay on the main stream) ends only when words[576] >= epoch, so the
 * mf_log_apply queued after it sees both groups' sums.  words: >= 1024 zeroed uint32 of device
 * memory owned by the caller, one per pair of streams (the arrival counters live there too);
 * epoch: increasing per chunk (wraps).  words[608] is set if a wait timed out (~0.4 s): the fold
 * is then invalid and the caller must fail.  words = NULL: no join. */
int mf_launch_join(void *words, int32_t role, uint32_t epoch);

/* mf_launch_fold(f): the chunk's fold (mf_log_apply, the same arithmetic and sum order) runs
 * inside the next mf_log_replay launch(es) of the calling thread instead of a launch of its own.
 * A piece's wave stores its sums through to the coherence point, then counts the piece in
 * item_count[item]; the wave that completes an item's pieces (over sums / item_piece_ptr and,
 * split chunk, sums2 / item_piece_ptr2 -- each group's replay is one launch, role 1 and 2 of
 * n_launches) applies that item.  No wave waits.  With stat_next, the last block of the
 * n_launches launches sums user_sq into it (mf_log_apply's <p^2> for the next chunk; fewer than
 * MF_SQ_PARTS_MIN users).  item_count: n_items zeroed int32 and words: MF_FOLD_WORDS zeroed
 * uint32, device memory owned by the caller (zero again after every complete fold).  Later
 * launches read q only after both replays have completed (the caller orders the streams).
 * Not with mf_launch_join.  f = NULL clears a pending fold.  Same fields as mf_log_apply (apply
 * = 1, no delta_out; hp read here, on the host). */
#define MF_FOLD_WORDS 1024
typedef struct mf_fold_t {
    void *qb;
    int32_t ld, n_factors, bias_col, rule;
    const void *sums;
    const int32_t *item_piece_ptr;
    const void *sums2;              /* nullable: one launch group */
    const int32_t *item_piece_ptr2;
    const int32_t *totals;
    const mf_hyper_t *hp;
    const double *p2stat;
    double *stat_next;              /* nullable */
    const double *user_sq;
    int64_t n_users;
    void *bias_out;                 /* nullable: the item-bias mirror */
    int32_t *item_count;
    uint32_t *words;
    int32_t role, n_launches;
} mf_fold_t;
int mf_launch_fold(const mf_fold_t *f);

#ifdef __cplusplus
}
#endif

#endif /* SURPRISE_AMD_H */
