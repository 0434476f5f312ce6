package io.sesam.dukemicroservice.gpu;

/**
 * A negative DK_E* status of libdukehip.so with its dk_last_error() text, thrown by every
 * DukeHip native.  An unchecked exception, so an uncaught one becomes HTTP 500 exactly as the
 * reference's DukeException does (App.java:1007-1009); GpuProcessor catches UNSUPPORTED to
 * hand the pipeline to stock Duke.
 */
public class DukeHipException extends RuntimeException {
    private static final long serialVersionUID = 1L;

    private final int code;

    public DukeHipException(int code, String message) {
        super("dukehip error " + code + ": " + message);
        this.code = code;
    }

    /** DukeHip.E_INVALID / E_UNSUPPORTED / E_NOMEM / E_DEVICE / E_STATE */
    public int code() {
        return code;
    }
}
