PFD = 2
exec(open("/root/repo/scripts/variants/cv_pf.py").read())
