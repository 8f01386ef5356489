//
// Drop-in public interface, declaration-identical to the reference's
// /root/reference/export_inc/IDecoder.h:15-41 (class IDecoder, vtable
// [dtor, deleting dtor, H265ToJpeg], static getInstance returning a new
// instance per call — not a singleton).
//

#ifndef H265TOJPEG_IDECODER_H
#define H265TOJPEG_IDECODER_H

#include <iostream>
#include <memory>

/**
 * Decoder interface: H.264/H.265 still -> JPEG.
 */
class IDecoder {

public:

    IDecoder() = default;

    virtual ~IDecoder() = default;

    /**
     * Decode the first picture of an H.264/H.265 Annex-B file and write it as JPEG.
     * @param inputFilePath  input H.264/H.265 file path
     * @param outputFilePath output JPEG file path
     * @return true on success
     */
    virtual bool H265ToJpeg(const char *inputFilePath, const char *outputFilePath) = 0;

    /**
     * A new decoder instance per call (NOT a singleton).
     */
    static std::shared_ptr<IDecoder> getInstance();
};

#endif //H265TOJPEG_IDECODER_H
