/*
 * spmv_rc.h — process exit / return codes of the MI355X SpMV suite.
 *
 * The numeric values are the reference's `ReturnCode` enum
 * (reference inc/enums.h:4-11) so scripts that test `$?` of ./bin/<fmt>
 * keep working.  The names drop "OpenCL": the device layer is HIP.
 */
#ifndef SPMV_RC_H
#define SPMV_RC_H

enum spmv_rc {
    SPMV_SUCCESS = 0,       /* reference Success            */
    SPMV_DEVICE_ERROR = 1,  /* reference OpenCLDeviceError  (no usable GPU / hipSetDevice failed) */
    SPMV_PROGRAM_ERROR = 2, /* reference OpenCLProgramError (alloc / copy / launch failed)        */
    SPMV_FILE_ERROR = 3,    /* reference FileError          (.mtx missing or rejected)             */
    SPMV_OTHER_ERROR = 4    /* reference OtherError         (bad arguments, unsupported config)    */
};

#endif /* SPMV_RC_H */
