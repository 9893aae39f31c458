"""Cut small slices of the reference's own fixture files (MNN tensor text format) into
tests/golden/: the first image row of SqueezeNet's C4 input and of MobileNet's quantised NHWC
input, token for token (data, not source).  Run here, where /root/reference exists."""
import os

REF = "/root/reference/execution-engine/resource/model"
OUT = os.path.dirname(os.path.abspath(__file__))


def tokens(path, n):
    out = []
    for line in open(path):
        out.extend(line.split())
        if len(out) >= n:
            return out[:n]
    return out


if __name__ == "__main__":
    # SqueezeNet input.txt: NC4HW4 [1][1][227][227][4]; the first row = 227 pixels x 4 lanes
    sq = tokens(f"{REF}/SqueezeNet/input.txt", 227 * 4)
    open(f"{OUT}/squeezenet_input_row0.txt", "w").write("\t".join(sq) + "\n")
    # MobileNet qnt_input.txt: NHWC [1][224][224][3]; the first row = 224 pixels x 3 channels
    mb = tokens(f"{REF}/MobileNet/qnt_input.txt", 224 * 3)
    open(f"{OUT}/mobilenet_qnt_input_row0.txt", "w").write(
        "".join("\t".join(mb[i:i + 3]) + "\t\n" for i in range(0, len(mb), 3)))
