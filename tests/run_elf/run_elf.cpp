// run.elf — test driver that restates the reference's CLI flow (src/main.cpp:16-99) against the
// MI355X drop-in library. TEST INFRASTRUCTURE: the CSR substrate that "stays" on the reference
// side (src/csr.cpp: reader, vectors, init_vector_rand, spmv_gold) is taken from the CPU
// oracle here (oracle/csr_ref.c), which is exactly what main.cpp links from csr.cpp; the
// hardware path is libspmv_hw (include/csr_hw_wrapper.h) with no CPU fallback.
//
// Usage: run.elf <matrix-file> [--fast-reader]   (env SPMV_NGPUS = units, like the reference's
// CU knob). --fast-reader reads the file with the library's Part-3 reader (spmv_read_csr_*,
// the drop-in for csr.cpp's read_csr_header / read_csr_matrix) instead of the oracle's, and
// prints the file read time.
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <sys/time.h>

#include "csr_hw_wrapper.h"

extern "C" {
int oracle_read_csr_header(const char *, IndexType *, IndexType *, IndexType *, IndexType, int *);
int oracle_read_csr_matrix(const char *, IndexType, IndexType, IndexType *, IndexType *, ValueType *);
void oracle_init_vector_rand(ValueType *, IndexType, ValueType);
void oracle_spmv_gold(IndexType, const IndexType *, const IndexType *, const ValueType *, const ValueType *,
                      ValueType *);
}

static double now_us()
{
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_usec + tv.tv_sec * 1e6;
}

int main(int argc, char **argv)
{
    const int units = spmv_hw_units();
#if DOUBLE == 0
    std::cout << "Welcome to SpMV (Compute Units : " << units << ", MI355X, single-precision arithmetic)\n";
#else
    std::cout << "Welcome to SpMV (Compute Units : " << units << ", MI355X, double-precision arithmetic)\n";
#endif
    const bool fast = argc == 3 && std::string(argv[2]) == "--fast-reader";
    if (argc != 2 && !fast) {
        std::printf("please enter the input file name  \n");
        return 1;
    }
    const double rd0 = now_us();
    csr_header hdr;
    if (fast ? spmv_read_csr_header(&hdr, argv[1])
             : oracle_read_csr_header(argv[1], &hdr.nr_rows, &hdr.nr_cols, &hdr.nr_nzeros, 32768, &hdr.blocks)) {
        std::cout << "Error reading matrix header\n";
        return 1;
    }
    csr_matrix matrix;
    matrix.nr_rows = hdr.nr_rows;
    matrix.nr_cols = hdr.nr_cols;
    matrix.nr_nzeros = hdr.nr_nzeros;
    matrix.row_ptr = (IndexType *)std::malloc((hdr.nr_rows + 1) * sizeof(IndexType));
    matrix.col_ind = (IndexType *)std::malloc((hdr.nr_nzeros + 1) * sizeof(IndexType));
    matrix.values = (ValueType *)std::malloc((hdr.nr_nzeros + 1) * sizeof(ValueType));
    matrix.Filename = argv[1];
    if (fast ? spmv_read_csr_matrix(&matrix, argv[1])
             : oracle_read_csr_matrix(argv[1], hdr.nr_rows, hdr.nr_nzeros, matrix.row_ptr, matrix.col_ind,
                                      matrix.values)) {
        std::cout << "Error reading matrix\n";
        return 1;
    }
    std::printf("File read time          : %.6f ms elapsed (%s reader)\n", (now_us() - rd0) / 1000,
                fast ? "spmv_read_csr" : "oracle");
    csr_vector x{(ValueType *)std::calloc(hdr.nr_cols + 1, sizeof(ValueType)), hdr.nr_cols};
    oracle_init_vector_rand(x.values, x.nr_values, 1);
    csr_vector y{(ValueType *)std::calloc(hdr.nr_rows + 1, sizeof(ValueType)), hdr.nr_rows};

    double s = now_us();
    oracle_spmv_gold(matrix.nr_rows, matrix.row_ptr, matrix.col_ind, matrix.values, x.values, y.values);
    std::printf("Software execution time : %.6f ms elapsed\n", (now_us() - s) / 1000);

    bool **empty_rows_bitmap;
    csr_hw_matrix **hw_matrix;
    csr_hw_vector *hw_x;
    s = now_us();
    create_csr_hw_matrix(&matrix, &hw_matrix, &empty_rows_bitmap);
    create_csr_hw_x_vector(&hw_x, &x, hw_matrix[0]->blocks, hw_matrix[0]->nr_cols);
    std::printf("Matrix read time        : %.6f ms elapsed\n", (now_us() - s) / 1000);

    csr_vector y_fpga{(ValueType *)std::calloc(hdr.nr_rows + 1, sizeof(ValueType)), hdr.nr_rows};
    spmv_hw(hw_matrix, hw_x, &y_fpga, empty_rows_bitmap);

    const int status = verification(y.nr_values, y.values, y_fpga.values, 0);
    std::cout << (status == 0 ? "Verification PASSED!\n" : "Verification FAILED!\n");

    ValueType mem = 0;
    const double csr_mem = ((matrix.nr_rows + 1.0) * INDEX_TYPE_BIT_WIDTH +
                            double(matrix.nr_nzeros) * (INDEX_TYPE_BIT_WIDTH + VALUE_TYPE_BIT_WIDTH)) /
                           (8.0 * 1024 * 1024);
    for (int i = 0; i < units; i++)
        mem += storage_overhead(hw_matrix[i]);
    std::cout << "CSR representation : " << csr_mem << " MB. Our representation : " << mem
              << " MB. Storage Overhead : " << (mem - csr_mem) / csr_mem * 100 << " %\n";

    delete_csr_hw_matrix(hw_matrix);
    std::free(empty_rows_bitmap);
    delete_csr_hw_x_vector(hw_x);
    std::free(matrix.row_ptr);
    std::free(matrix.col_ind);
    std::free(matrix.values);
    std::free(x.values);
    std::free(y.values);
    std::free(y_fpga.values);
    return status;
}
