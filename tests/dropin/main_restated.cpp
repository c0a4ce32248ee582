// tests/dropin/main_restated.cpp — TEST INFRASTRUCTURE: the reference CLI's include list and call
// sequence (src/main.cpp:1-99), restated, built against include/dropin/ exactly as an unchanged
// main.cpp would be: <sds_lib.h>, "util.h", "csr.h", "csr_hw.h", "csr_hw_wrapper.h", "spmv.h"
// (main.cpp:8-14), a compile-time ComputeUnits loop over hw_matrix (main.cpp:86-87) and
// free() of the bitmap's outer array (main.cpp:95). Prints the library's unit count and the sum
// of storage_overhead over the ComputeUnits slots so the test can check them.
#include <iostream>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <math.h>
#include <string>

#include <sds_lib.h>

#include "util.h"
#include "csr.h"
#include "csr_hw.h"
#include "csr_hw_wrapper.h"
#include "spmv.h"

int main(int argc, char **argv)
{
    std::cout << "Drop-in build: CU " << ComputeUnits << ", library units " << spmv_hw_units() << "\n";
    if (argc != 2) {
        printf("please enter the input file name  \n");
        return 1;
    }
    csr_header hdr;
    if (read_csr_header(&hdr, argv[1]) != 0) {
        std::cout << "Error reading matrix header\n";
        return 1;
    }
    csr_matrix *A = create_csr_matrix(hdr);
    if (read_csr_matrix(A, argv[1]) != 0) {
        std::cout << "Error reading matrix\n";
        return 1;
    }
    csr_vector *x = create_csr_vector(hdr.nr_cols);
    init_vector_rand(x, 1);
    csr_vector *y_ref = create_csr_vector(hdr.nr_rows);
    double t = getTimestamp();
    spmv_gold(A, x->values, y_ref->values);
    printf("Software execution time : %.6f ms elapsed\n", (getTimestamp() - t) / 1000);

    bool **bitmap;
    csr_hw_matrix **hw;
    csr_hw_vector *hx;
    t = getTimestamp();
    create_csr_hw_matrix(A, &hw, &bitmap);
    create_csr_hw_x_vector(&hx, x, hw[0]->blocks, hw[0]->nr_cols);
    printf("Matrix read time        : %.6f ms elapsed\n", (getTimestamp() - t) / 1000);

    csr_vector *y_hw = create_csr_vector(hdr.nr_rows);
    spmv_hw(hw, hx, y_hw, bitmap);
    // IndexType by value: the caller-typed overload of the drop-in header
    const int status = verification(y_ref->nr_values, y_ref->values, y_hw->values, 0);
    std::cout << (status == 0 ? "Verification PASSED!\n" : "Verification FAILED!\n");

    // every slot up to the compile-time ComputeUnits, whatever the library's unit count
    ValueType mem = 0;
    int nonnull = 0;
    for (int i = 0; i < ComputeUnits; i++) {
        mem += storage_overhead(hw[i]);
        nonnull += hw[i] != NULL;
    }
    printf("storage_overhead over %d ComputeUnits slots: %.6f MB, %d non-null handles\n", ComputeUnits,
           (double)mem, nonnull);

    void *scratch = sds_alloc(4096);  // the SDSoC allocator of <sds_lib.h> still links
    sds_free(scratch);

    delete_csr_matrix(A);
    delete_csr_vector(x);
    delete_csr_vector(y_ref);
    delete_csr_hw_matrix(hw);
    free(bitmap);
    delete_csr_hw_x_vector(hx);
    delete_csr_vector(y_hw);
    return status;
}
