/*
 * ref_ocl_runner.c -- runs the REFERENCE OpenCL kernel (raytracer_bvh,
 * x64/Release/volumeRender.cl) on the GPU through the ROCm OpenCL runtime.
 *
 * TEST INFRASTRUCTURE ONLY (oracle pin).  The kernel code object
 * is compiled from the reference source where it lies by oracle/Makefile.ref
 * into oracle/_ref/ (git-ignored); this file is this repository's own host
 * harness.  It reproduces the reference host's argument binding
 * (RayTracer.cpp:1222-1261), buffer creation (RayTracer.cpp:942-984) and
 * launch shape (RayTracer.cpp:330-344: 2-D NDRange rounded up to 8x8
 * work-groups, clFinish, blocking read).
 */
#define CL_TARGET_OPENCL_VERSION 120
#include <CL/cl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void err(char* buf, int len, const char* what, cl_int e) {
    if (buf && len > 0) snprintf(buf, (size_t)len, "%s failed (%d)", what, (int)e);
}

static size_t round_up(size_t loc, size_t w) { return (w / loc + (w % loc > 0 ? 1 : 0)) * loc; }

int refocl_device_count(void) {
    cl_platform_id plats[8];
    cl_uint np = 0, total = 0;
    if (clGetPlatformIDs(8, plats, &np) != CL_SUCCESS) return 0;
    for (cl_uint i = 0; i < np; ++i) {
        cl_uint nd = 0;
        if (clGetDeviceIDs(plats[i], CL_DEVICE_TYPE_GPU, 0, NULL, &nd) == CL_SUCCESS) total += nd;
    }
    return (int)total;
}

/* Returns 0 on success.  params: 32 floats (Params, RayTracer.cpp:115-161). */
int refocl_render(const char* binary_path, const float* params, const float* verts, int nv, const int* idx,
                  int nidx, const void* nodes, int nn, const int* refs, int nref, const float* normals, int nnorm,
                  const int* nidx_arr, const void* mats, int nmat, const int* tri2mat, uint32_t w, uint32_t h,
                  uint32_t* out, char* errbuf, int errlen) {
    cl_int e;
    cl_platform_id plats[8];
    cl_uint np = 0;
    cl_device_id dev = NULL;
    int rc = -1;
    FILE* f = fopen(binary_path, "rb");
    if (!f) { if (errbuf) snprintf(errbuf, errlen, "cannot open %s", binary_path); return -1; }
    fseek(f, 0, SEEK_END);
    long bl = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* bin = (unsigned char*)malloc((size_t)bl);
    if (!bin || fread(bin, 1, (size_t)bl, f) != (size_t)bl) { fclose(f); free(bin); return -1; }
    fclose(f);

    if ((e = clGetPlatformIDs(8, plats, &np)) != CL_SUCCESS || np == 0) { err(errbuf, errlen, "clGetPlatformIDs", e); free(bin); return -1; }
    for (cl_uint i = 0; i < np && !dev; ++i) clGetDeviceIDs(plats[i], CL_DEVICE_TYPE_GPU, 1, &dev, NULL);
    if (!dev) { err(errbuf, errlen, "no OpenCL GPU device", 0); free(bin); return -1; }
    cl_context ctx = clCreateContext(NULL, 1, &dev, NULL, NULL, &e);
    if (e != CL_SUCCESS) { err(errbuf, errlen, "clCreateContext", e); free(bin); return -1; }
    cl_command_queue q = clCreateCommandQueue(ctx, dev, 0, &e);
    const size_t blen = (size_t)bl;
    const unsigned char* bp = bin;
    cl_int bstat = 0;
    cl_program prog = clCreateProgramWithBinary(ctx, 1, &dev, &blen, &bp, &bstat, &e);
    free(bin);
    cl_kernel k = NULL;
    cl_mem bufs[12] = {0};
    if (e != CL_SUCCESS) { err(errbuf, errlen, "clCreateProgramWithBinary", e); goto done; }
    if ((e = clBuildProgram(prog, 1, &dev, "", NULL, NULL)) != CL_SUCCESS) { err(errbuf, errlen, "clBuildProgram", e); goto done; }
    k = clCreateKernel(prog, "raytracer_bvh", &e);
    if (e != CL_SUCCESS) { err(errbuf, errlen, "clCreateKernel", e); goto done; }
    {
        const cl_mem_flags RO = CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR;
        cl_mem out_b = bufs[0] = clCreateBuffer(ctx, CL_MEM_WRITE_ONLY, (size_t)w * h * 4, NULL, &e);
        cl_mem par_b = bufs[1] = clCreateBuffer(ctx, RO, 128, (void*)params, &e);
        cl_mem v_b = bufs[2] = clCreateBuffer(ctx, RO, (size_t)nv * 16, (void*)verts, &e);
        cl_mem i_b = bufs[3] = clCreateBuffer(ctx, RO, (size_t)nidx * 4, (void*)idx, &e);
        cl_mem n_b = bufs[4] = clCreateBuffer(ctx, RO, (size_t)nn * 48, (void*)nodes, &e);
        cl_mem r_b = bufs[5] = clCreateBuffer(ctx, RO, (size_t)(nref > 0 ? nref : 1) * 4, (void*)refs, &e);
        cl_mem t_b = bufs[6] = clCreateBuffer(ctx, CL_MEM_WRITE_ONLY, (64 + 1) * 16, NULL, &e);
        cl_mem nm_b = bufs[7] = clCreateBuffer(ctx, RO, (size_t)nnorm * 16, (void*)normals, &e);
        cl_mem ni_b = bufs[8] = clCreateBuffer(ctx, RO, (size_t)nidx * 4, (void*)nidx_arr, &e);
        cl_mem m_b = bufs[9] = clCreateBuffer(ctx, RO, (size_t)nmat * 176, (void*)mats, &e);
        cl_mem tm_b = bufs[10] = clCreateBuffer(ctx, RO, (size_t)(nidx / 3) * 4, (void*)tri2mat, &e);
        cl_mem null_b = NULL;
        int zero = 0;
        e = 0;
        e |= clSetKernelArg(k, 0, sizeof(cl_mem), &out_b);
        e |= clSetKernelArg(k, 1, sizeof(unsigned int), &w);
        e |= clSetKernelArg(k, 2, sizeof(unsigned int), &h);
        e |= clSetKernelArg(k, 3, sizeof(cl_mem), &null_b);
        e |= clSetKernelArg(k, 4, sizeof(cl_int), &zero);
        e |= clSetKernelArg(k, 5, sizeof(cl_mem), &par_b);
        e |= clSetKernelArg(k, 6, sizeof(cl_mem), &v_b);
        e |= clSetKernelArg(k, 7, sizeof(cl_mem), &i_b);
        e |= clSetKernelArg(k, 8, sizeof(cl_mem), &n_b);
        e |= clSetKernelArg(k, 9, sizeof(cl_mem), &r_b);
        e |= clSetKernelArg(k, 10, sizeof(cl_int), &nref);
        e |= clSetKernelArg(k, 11, sizeof(cl_int), &nn);
        e |= clSetKernelArg(k, 12, sizeof(cl_mem), &t_b);
        e |= clSetKernelArg(k, 13, sizeof(cl_mem), &nm_b);
        e |= clSetKernelArg(k, 14, sizeof(cl_mem), &ni_b);
        e |= clSetKernelArg(k, 15, sizeof(cl_mem), &m_b);
        e |= clSetKernelArg(k, 16, sizeof(cl_mem), &tm_b);
        if (e != CL_SUCCESS) { err(errbuf, errlen, "clSetKernelArg", e); goto done; }
        const size_t local_ws[2] = {8, 8};
        const size_t global_ws[2] = {round_up(8, w), round_up(8, h)};
        if ((e = clEnqueueNDRangeKernel(q, k, 2, NULL, global_ws, local_ws, 0, NULL, NULL)) != CL_SUCCESS) { err(errbuf, errlen, "clEnqueueNDRangeKernel", e); goto done; }
        if ((e = clFinish(q)) != CL_SUCCESS) { err(errbuf, errlen, "clFinish", e); goto done; }
        if ((e = clEnqueueReadBuffer(q, out_b, CL_TRUE, 0, (size_t)w * h * 4, out, 0, NULL, NULL)) != CL_SUCCESS) { err(errbuf, errlen, "clEnqueueReadBuffer", e); goto done; }
        rc = 0;
    }
done:
    for (int i = 0; i < 12; ++i) if (bufs[i]) clReleaseMemObject(bufs[i]);
    if (k) clReleaseKernel(k);
    if (prog) clReleaseProgram(prog);
    if (q) clReleaseCommandQueue(q);
    clReleaseContext(ctx);
    return rc;
}
