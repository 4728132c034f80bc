"""Python stand-in for the R package's runner.R (R/R/cluster.R spark_apply), used to test
the R barrier launch path without R: same command line (dir, on_error mode, rank), same
result protocol (result-<rank>.json ~ result-<rank>.rds: {ok, value}), same exit status on
an error in "restart" mode.  The "closure" is picked by DAMD_SHIM_BEHAVIOUR."""
import json
import os
import sys
import time


def closure(i, barrier, attempt):
    how = os.environ.get("DAMD_SHIM_BEHAVIOUR", "ok")
    if how == "crash1" and i == 1 and attempt == 0:
        os._exit(9)  # a hard worker crash (not an R error)
    if how == "hang0" and i == 0 and attempt == 0:
        time.sleep(3600)  # a survivor that would hold its GPU forever
    if how == "error1" and i == 1:
        raise ValueError("boom in partition 1")
    return f"{barrier['partition']}/{len(barrier['address'])}/attempt{attempt}"


def main():
    d, mode, i = sys.argv[1], sys.argv[2], int(sys.argv[3])
    addr = open(os.path.join(d, "addresses.txt")).read().split()
    attempt = int(os.environ.get("DAMD_RESTART_COUNT", "0"))
    if os.environ.get("DAMD_SHIM_BEHAVIOUR") == "crash1+hang0" and i == 0 and attempt == 0:
        time.sleep(3600)
    if os.environ.get("DAMD_SHIM_BEHAVIOUR") == "crash1+hang0" and i == 1 and attempt == 0:
        time.sleep(0.5)
        os._exit(9)
    try:
        res = {"ok": True, "value": closure(i, {"address": addr, "partition": i}, attempt)}
    except Exception as e:  # tryCatch(..., error = function(e) conditionMessage(e))
        res = {"ok": False, "value": str(e)}
    with open(os.path.join(d, f"result-{i}.json"), "w") as f:
        json.dump(res, f)
    if not res["ok"] and mode == "restart":
        sys.exit(3)


if __name__ == "__main__":
    main()
