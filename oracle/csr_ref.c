/*
 * oracle/csr_ref.c — CPU restatement of the reference's SpMV path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg and the test driver
 * tests/run_elf may load this code, and only as the checker (or the timed CPU baseline).
 * The product library (spmv-fpga_amd/) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned". The reference (euroexa/spmv-fpga) cannot be built in this
 * image: every source includes Xilinx ap_int.h / hls_stream.h / sds_lib.h (util.h:7,
 * spmv.cpp:2, csr_hw.h:5, main.cpp:8), which are not installed, and building it with
 * stand-ins is not allowed. The reference ships no tests, fixtures or golden vectors
 * (SURVEY.md §4). What pins this restatement instead (tests/test_oracle.py):
 *   - glibc rand() known answers for init_vector_rand recorded in SURVEY.md §8(a3);
 *   - an independent numpy restatement of spmv_gold, bit-exact on every fixture;
 *   - the reference's own self-check (main.cpp:77-82): the restated FPGA arithmetic order
 *     (spmv.cpp:66-104 + csr_hw.cpp:1531-1565) must pass verification (abs 1e-5) against
 *     spmv_gold on every fixture, for every valid (CU, VF);
 *   - the only known answers the reference itself holds, its diagrams (images/1_matrix.svg,
 *     2_csr.svg, 3_hw_representation_v3.svg, transcribed into
 *     tests/golden/reference_diagram_kat.json): the reader gives the diagram's CSR and the
 *     restated packed format (oracle.py pack_hw_submatrix) gives its bus words.
 *
 * Build: gcc -O2 -ffp-contract=off (no FMA, like the reference's -O2 build without -march),
 * -DDOUBLE=1 -> liboracle_f64.so, -DDOUBLE=0 -> liboracle_f32.so (oracle/Makefile).
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <math.h>

#ifndef DOUBLE
#define DOUBLE 1
#endif

typedef uint32_t IndexType;
#if DOUBLE == 0
typedef float ValueType;
#define LINE_FMT "%u %u %f"
#else
typedef double ValueType;
#define LINE_FMT "%u %u %lf"
#endif

int oracle_value_bytes(void) { return (int)sizeof(ValueType); }

/* csr.cpp:10-46 — header line "rows cols nnz"; blocks = ceil(cols / cols_div_blocks). */
int oracle_read_csr_header(const char *path, IndexType *nr_rows, IndexType *nr_cols,
                           IndexType *nr_nzeros, IndexType cols_div_blocks, int *blocks)
{
    FILE *fp = fopen(path, "r");
    if (!fp)
        return 1;
    int matched = fscanf(fp, "%u %u %u\n", nr_rows, nr_cols, nr_nzeros);
    fclose(fp);
    if (matched == EOF)
        return 1;
    if (matched != 3)
        return 3;
    if (blocks) {
        int b = (int)(*nr_cols / cols_div_blocks) + 1;
        if (*nr_cols % cols_div_blocks == 0)
            b--;
        *blocks = b;
    }
    return 0;
}

/* csr.cpp:87-136. Entries "r c v" are 1-based and sorted by row; empty rows get the running
 * count (csr.cpp:115-116); row_ptr[n] = header nnz (csr.cpp:126). Deviation: rows
 * after the last entry are filled too, where the reference leaves them uninitialised. */
int oracle_read_csr_matrix(const char *path, IndexType nr_rows, IndexType nr_nzeros,
                           IndexType *row_ptr, IndexType *col_ind, ValueType *values)
{
    char line[1000];
    FILE *fp = fopen(path, "r");
    if (!fp)
        return 1;
    if (!fgets(line, sizeof line, fp)) {
        fclose(fp);
        return 1;
    }
    IndexType row_ptr_pos = 0, values_pos = 0;
    while (fgets(line, sizeof line, fp) != NULL) {
        IndexType r, c;
        ValueType v;
        if (sscanf(line, LINE_FMT, &r, &c, &v) != 3) {
            fclose(fp);
            return 1;
        }
        if (values_pos >= nr_nzeros || r < 1 || r > nr_rows || r < row_ptr_pos) {
            fclose(fp);
            return 4; /* more entries than the header says, or rows not sorted */
        }
        for (IndexType i = row_ptr_pos; i < r; i++)
            row_ptr[i] = values_pos;
        row_ptr_pos = r;
        col_ind[values_pos] = c - 1;
        values[values_pos] = v;
        values_pos++;
    }
    for (IndexType i = row_ptr_pos; i < nr_rows; i++) /* B2 fix: trailing empty rows */
        row_ptr[i] = values_pos;
    row_ptr[nr_rows] = nr_nzeros;
    int err = ferror(fp) ? 2 : 0;
    fclose(fp);
    return err;
}

/* csr.cpp:170-179 with the libc generator. The reference never calls srand (seed 1). */
void oracle_srand(unsigned seed) { srand(seed); }
void oracle_init_vector_rand(ValueType *x, IndexType n, ValueType max)
{
    for (IndexType i = 0; i < n; i++)
        x[i] = max * (rand() / (ValueType)RAND_MAX);
}

/* csr.cpp:184-194: per row, accumulate in ValueType from 0.0 in CSR order, then store. */
void oracle_spmv_gold(IndexType nr_rows, const IndexType *row_ptr, const IndexType *col_ind,
                      const ValueType *values, const ValueType *x, ValueType *y)
{
    for (IndexType i = 0; i < nr_rows; i++) {
        ValueType acc = 0.0;
        for (IndexType j = row_ptr[i]; j < row_ptr[i + 1]; j++)
            acc += values[j] * x[col_ind[j]];
        y[i] = acc;
    }
}

/* spmv_gold's products (csr.cpp:190: val * x rounded to ValueType) summed in fp64 from 0 in
 * CSR order, rounded to ValueType once per row. Not a reference function: it is the checker
 * for the GPU kernels that accumulate fp32 products in fp64 (sweep, binned, slices): against it
 * their error is fp64 reassociation only, so a tight bound holds where spmv_gold's own fp32
 * running sum (over a 2M-entry row, say) is the less accurate side. Identical to spmv_gold for
 * fp64. */
void oracle_spmv_fp64acc(IndexType nr_rows, const IndexType *row_ptr, const IndexType *col_ind,
                         const ValueType *values, const ValueType *x, ValueType *y)
{
    for (IndexType i = 0; i < nr_rows; i++) {
        double acc = 0.0;
        for (IndexType j = row_ptr[i]; j < row_ptr[i + 1]; j++) {
            const ValueType prod = values[j] * x[col_ind[j]];
            acc += (double)prod;
        }
        y[i] = (ValueType)acc;
    }
}

/* Same arithmetic on a contiguous row range, for timing a bounded CPU sample. */
void oracle_spmv_gold_rows(IndexType row_begin, IndexType row_end, const IndexType *row_ptr,
                           const IndexType *col_ind, const ValueType *values, const ValueType *x,
                           ValueType *y)
{
    for (IndexType i = row_begin; i < row_end; i++) {
        ValueType acc = 0.0;
        for (IndexType j = row_ptr[i]; j < row_ptr[i + 1]; j++)
            acc += values[j] * x[col_ind[j]];
        y[i - row_begin] = acc;
    }
}

/* Arithmetic order of the reference FPGA path, per row:
 *   column blocks of `cols_div_blocks` columns (csr_hw.cpp:25-27,64-76); within block b the
 *   row's elements in CSR order (create_block_matrix, csr_hw.cpp:209-243), zero-padded to a
 *   multiple of VF (:228-238); compute_results (spmv.cpp:74-103) sums each VF group from 0
 *   left to right and adds the group to the running row sum; accum_results
 *   (csr_hw.cpp:1543-1562, loop csr_hw_wrapper.cpp:276-281) adds each block's row sum into the
 *   caller's y in block order. y is ACCUMULATED (+=), like spmv_hw.
 * The CU partition (prepare_balanced_hw_matrix) never splits a row inside a block, so it does
 * not change any row's arithmetic; it is not restated. x beyond nr_cols reads the zero padding
 * of write_csr_hw_vector (csr_hw.cpp:1478-1484). */
void oracle_spmv_fpga_order(IndexType nr_rows, IndexType nr_cols, const IndexType *row_ptr,
                            const IndexType *col_ind, const ValueType *values, const ValueType *x,
                            ValueType *y, IndexType cols_div_blocks, int vf)
{
    int blocks = (int)(nr_cols / cols_div_blocks) + 1;
    if (nr_cols % cols_div_blocks == 0)
        blocks--;
    for (int b = 0; b < blocks; b++) {
        IndexType lo = (IndexType)b * cols_div_blocks;
        IndexType hi = (b == blocks - 1) ? 0xFFFFFFFFu : lo + cols_div_blocks - 1;
        ValueType pad_x = (lo < nr_cols) ? x[lo] : (ValueType)0; /* padded entries use col 0 */
        for (IndexType i = 0; i < nr_rows; i++) {
            ValueType sum = 0;
            ValueType group = 0;
            int in_group = 0, count = 0;
            for (IndexType j = row_ptr[i]; j < row_ptr[i + 1]; j++) {
                IndexType c = col_ind[j];
                if (c < lo || c > hi)
                    continue;
                ValueType xv = (c < nr_cols) ? x[c] : (ValueType)0;
                group += values[j] * xv;
                count++;
                if (++in_group == vf) {
                    sum += group;
                    group = 0;
                    in_group = 0;
                }
            }
            if (count == 0)
                continue; /* empty in this block: bitmap entry set, y untouched */
            if (in_group != 0) {
                for (; in_group < vf; in_group++)
                    group += (ValueType)0 * pad_x;
                sum += group;
            }
            y[i] += sum;
        }
    }
}

/* Test metric only (not in the reference): (|A||x|)_i in fp64, the denominator of the parity
 * tests' componentwise-scaled error. */
void oracle_abs_spmv(IndexType nr_rows, const IndexType *row_ptr, const IndexType *col_ind,
                     const ValueType *values, const ValueType *x, double *out)
{
    for (IndexType i = 0; i < nr_rows; i++) {
        double acc = 0.0;
        for (IndexType j = row_ptr[i]; j < row_ptr[i + 1]; j++)
            acc += fabs((double)values[j]) * fabs((double)x[col_ind[j]]);
        out[i] = acc;
    }
}

/* csr_hw.cpp:1571-1590: error when |sw - hw| >= 1e-5 or NaN. Returns the error count. */
long oracle_verification_errors(IndexType n, const ValueType *sw, const ValueType *hw)
{
    const ValueType thres = (ValueType)1e-5;
    long errors = 0;
    for (IndexType i = 0; i < n; i++) {
        ValueType diff = (ValueType)fabs((double)(sw[i] - hw[i]));
        if (diff >= thres || diff != diff)
            errors++;
    }
    return errors;
}
